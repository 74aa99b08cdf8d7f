# Critical-path FedAvg through RCCL: on the compute stream (default) vs the side stream
# (MYFYP_FEDAVG_SIDE=1), one-peer and two-peer loads, arms alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6n_fedavg_stream_ab; mkdir -p $O
b() { timeout -k 10 200 python bench.py --peers $1 --n-train $((7500 * $1)) --n-test $((1250 * $1)) --steps 200 --warmup 10 --force-collective; }
for i in 1 2 3; do
  MYFYP_FEDAVG_SIDE=1 b 1 > $O/side_p1_$i.log 2>&1 || exit 1
  b 1 > $O/cur_p1_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  MYFYP_FEDAVG_SIDE=1 b 2 > $O/side_p2_$i.log 2>&1 || exit 1
  b 2 > $O/cur_p2_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
