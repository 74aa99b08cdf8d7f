#!/bin/bash
# round 4, call X: halo dgrad epilogue operands loaded before the tile MFMAs (EPI_PF_HALO): CNN tests,
# ResNet-18 A/B, windowed kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4x; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-200; case $rc in 0) ;; *) exit $rc;; esac; }
run test_cnn 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_engine_gpu.py
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
run rn_new_a 300 $R
MYFYP_NATIVE_LIB=build/ab_EPI_PF_HALO0/libmyfyp_hip.so run rn_old_a 300 $R
run rn_new_b 300 $R
MYFYP_NATIVE_LIB=build/ab_EPI_PF_HALO0/libmyfyp_hip.so run rn_old_b 300 $R
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 5 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/tools/rocpd_window_stats.py "$T" k_opt_step 0 > $O/resnet_window_stats.csv 2> $O/window.txt && cat $O/window.txt && head -16 $O/resnet_window_stats.csv | cut -c1-150
rm -f "$T"
