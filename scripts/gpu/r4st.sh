#!/bin/bash
# round 4, call ST: the 64-column LDS-DMA forward (ResNet-18 stem) with compile-time epilogue operand
# sets: CNN tests, ResNet-18 10 rounds, windowed kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4st; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-160; case $rc in 0) ;; *) exit $rc;; esac; }
run test_cnn 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_cnn_engine_gpu.py
run rn_a 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 5 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/tools/rocpd_window_stats.py "$T" k_opt_step 0 > $O/resnet_window_stats.csv 2> $O/window.txt && cat $O/window.txt && grep "128, 64" $O/resnet_window_stats.csv | cut -c1-150
rm -f "$T"
