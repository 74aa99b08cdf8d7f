# Same-box check of the ResNet-18 round rate against the round-5 tree (git worktree _abtree at
# 643758b, built in-tree), arms alternating; then the MLP per-GPU loads (r6h_mlp_loads.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6i_vs_r5; mkdir -p $O
for i in 1 2; do
  (cd _abtree && timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/r5_$i.log 2>&1) || exit 1
  timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/r6_$i.log 2>&1 || exit 1
done
for f in $O/r5_*.log $O/r6_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["round_ms_per_local_step"])')"; done
bash scripts/gpu/r6h_mlp_loads.sh
