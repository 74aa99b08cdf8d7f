# ResNet-18 (config 4) A/B: halo wgrad prefetch depth 1 vs 2 (the new default), alternating arms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6e_resnet_pf; mkdir -p $O
for i in 1 2; do
  MYFYP_WGRAD_PF=1 timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/pf1_$i.log 2>&1 || exit 1
  timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/pf2_$i.log 2>&1 || exit 1
done
for f in $O/pf*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_round"])')"; done
