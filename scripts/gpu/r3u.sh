#!/bin/bash
# round 3, call U: gang commit before the fp32 epoch's write-back: fp32 MLP + kernel tests, bench x2
set -o pipefail
O=gpurun_out/r3x_u; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_kernels_gpu.py tests/test_multiproc_gpu.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed" >> $O/status; exit 1; }
for i in 1 2; do timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_$i.log 2>&1 || exit 1; done
echo done >> $O/status
