#!/bin/bash
# round 4, call J: result ring by sequence word (no event record behind each publish) and lazy gang-order
# event: MLP GPU tests, round timeline, bench A/B against the old event path
set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -4 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
run test_mlp 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py tests/test_kernels_gpu.py tests/test_collective_gpu.py tests/test_rccl_forced_gpu.py
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cat $O/timeline.txt | cut -c1-120
rm -f "$D"
run bench_new_a 200 python bench.py --steps 200 --warmup 10
MYFYP_RING_EVENTS=1 MYFYP_GANG_EVENT=1 run bench_old_a 200 python bench.py --steps 200 --warmup 10
run bench_new_b 200 python bench.py --steps 200 --warmup 10
MYFYP_RING_EVENTS=1 MYFYP_GANG_EVENT=1 run bench_old_b 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=2 run bench_new_prep2 200 python bench.py --steps 200 --warmup 10
