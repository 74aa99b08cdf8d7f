#!/bin/bash
# round 3, call C: synthetic CIFAR difficulty sweep (LeNet ring, ResNet FedAvg) + rebalanced fp32 MLP kernel
set -o pipefail
O=gpurun_out/r3x_c; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 240 --timeout-method thread > $O/mlp_f32_tests.log 2>&1; echo "mlp_f32 tests rc=$?" >> $O/status
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_plain.log 2>&1 || exit 1
i=0
for cfg in "0.75 1.0 2 0.1" "0.8 1.2 4 0.1" "0.85 1.2 4 0.1" "0.7 1.2 4 0.05" "0.8 1.0 4 0.0"; do
  set -- $cfg; i=$((i+1))
  timeout -k 10 200 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 2 --similarity $1 --noise $2 --modes $3 --label-noise $4 > $O/lenet_$i.log 2>&1 || exit 1
done
i=0
for cfg in "0.75 1.0 2 0.1" "0.8 1.2 4 0.1" "0.7 1.2 4 0.05"; do
  set -- $cfg; i=$((i+1))
  timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1 --similarity $1 --noise $2 --modes $3 --label-noise $4 > $O/resnet_$i.log 2>&1 || exit 1
done
