#!/bin/bash
# round 3, call A: forced-collective RCCL path + benches + kernel trace
set -o pipefail
O=gpurun_out/r3x_a; mkdir -p $O
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_rccl_forced_gpu.py -x -v --timeout 480 --timeout-method thread > $O/forced_test.log 2>&1; echo "forced_test rc=$?" >> $O/status
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_plain.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 200 --warmup 10 --force-collective > $O/bench_forced.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 200 --warmup 10 --force-collective --no-failover > $O/bench_forced_nofo.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_forced -o run -- python3 bench.py --steps 30 --warmup 5 --force-collective > $O/prof_forced.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "pytest_gpu rc=$?" >> $O/status
