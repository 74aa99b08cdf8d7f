#!/bin/bash
# GPU tests (all) + headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -4 gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log; grep '^\[bench\]' gpurun_out/bench1.log
