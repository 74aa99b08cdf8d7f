#!/bin/bash
# round 3, call R: unfenced C2 default: tests, stamps, bench x3
set -o pipefail
O=gpurun_out/r3x_r; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed" >> $O/status; exit 1; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 120 python scripts/probes/stamps_f32.py > $O/stamps.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_$i.log 2>&1 || exit 1; done
echo done >> $O/status
