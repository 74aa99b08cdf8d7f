#!/bin/bash
# round 5: headline round boundary — direct epoch launch and snapshot wait-by-value, A/B + tests + timeline
set -o pipefail
O=gpurun_out/r5_bnd; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-200; case $rc in 0) ;; *) exit $rc;; esac; }
run tests 400 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_kernels_gpu.py tests/test_device_mesh_gpu.py -x -q --timeout 120 --timeout-method thread
for k in a b; do
run bench_new_$k 200 python bench.py --steps 200 --warmup 10
MYFYP_EPOCH_GRAPH=1 MYFYP_SNAP_EVENT=1 run bench_old_$k 200 python bench.py --steps 200 --warmup 10
MYFYP_EPOCH_GRAPH=1 run bench_graph_$k 200 python bench.py --steps 200 --warmup 10
MYFYP_SNAP_EVENT=1 run bench_event_$k 200 python bench.py --steps 200 --warmup 10
done
run bench20 200 python bench.py --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-140 $O/timeline.txt | tail -14
rm -f "$D"
