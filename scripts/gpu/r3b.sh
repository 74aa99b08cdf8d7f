#!/bin/bash
# round 3, call B: forced RCCL test, lag-one failover cost, async CNN round, CIFAR difficulty calibration
set -o pipefail
O=gpurun_out/r3x_b; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_rccl_forced_gpu.py tests/test_multiproc_gpu.py tests/test_cnn_engine_gpu.py -x -v --timeout 480 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/status
timeout -k 10 120 python bench.py --steps 200 --warmup 10 --force-collective > $O/bench_forced_fo.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_plain.log 2>&1 || exit 1
timeout -k 10 200 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 > $O/lenet_ring.log 2>&1 || exit 1
timeout -k 10 200 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 --similarity 0.6 --noise 1.0 --modes 1 --label-noise 0 > $O/lenet_ring_easy.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1 > $O/resnet_fedavg.log 2>&1 || exit 1
