#!/bin/bash
# round 4, call L: (1) fit results published by the epoch graph's last node + double-buffered evaluation
# sides (host-side wait): MLP GPU tests, round timeline, bench A/B; (2) call K's CNN work (halo dgrad
# with DMA-staged patches)
set -o pipefail
O=gpurun_out/r4l; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
run test_mlp 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py tests/test_collective_gpu.py tests/test_kernels_gpu.py
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-120 $O/timeline.txt
rm -f "$D"
run bench_a 200 python bench.py --steps 200 --warmup 10
MYFYP_GRAPH_PUBLISH=0 run bench_nogp_a 200 python bench.py --steps 200 --warmup 10
run bench_b 200 python bench.py --steps 200 --warmup 10
MYFYP_GRAPH_PUBLISH=0 run bench_nogp_b 200 python bench.py --steps 200 --warmup 10
bash scripts/gpu/r4k.sh
