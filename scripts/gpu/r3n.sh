#!/bin/bash
# round 3, call N: stride-1 dgrad as a forward conv (MODE 4): numerics, per-layer timings, ResNet A/B
set -o pipefail
O=gpurun_out/r3x_n; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -x -v --timeout 200 --timeout-method thread > $O/cnn_tests.log 2>&1 || { echo "cnn tests failed" >> $O/status; exit 1; }
timeout -k 10 120 python scripts/probes/conv_ab.py > $O/conv_ab.log 2>&1 || exit 1
for i in 1 2; do
  MYFYP_DGRAD_FWD=1 timeout -k 10 240 python benchmarks/bench_cnn.py --model resnet18 --rounds 4 --warmup 1 > $O/resnet_m4_$i.log 2>&1 || exit 1
  MYFYP_DGRAD_FWD=0 timeout -k 10 240 python benchmarks/bench_cnn.py --model resnet18 --rounds 4 --warmup 1 > $O/resnet_m3_$i.log 2>&1 || exit 1
done
echo done >> $O/status
