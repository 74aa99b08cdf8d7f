# One peer per device: is the fp32 epoch exact at every K split? Probe (per-parameter errors vs torch,
# no extras) at K split 1 / 2 / 4 / 8 with one and two peers, and the one-peer bench's accuracy at
# K split 1 vs the cross-XCD K split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6q_p1_correct; mkdir -p $O
PEERS=1 timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 1,2,4,8 > $O/probe_p1.log 2>&1 || exit 1
PEERS=3 timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 4 > $O/probe_p3.log 2>&1 || exit 1
grep -h "extra=False" $O/probe_*.log
b() { timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --n-test 1250 --steps 100 --warmup 5; }
MYFYP_F32_XSPLIT=0 b > $O/bench_p1_ks1.log 2>&1 || exit 1
b > $O/bench_p1_xr.log 2>&1 || exit 1
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["final_test_acc"], d["rounds_to_target"], d["config"]["engine"])')"; done
