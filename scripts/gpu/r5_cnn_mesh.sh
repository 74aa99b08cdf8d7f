set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_cnn_mesh; mkdir -p $O
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --gpus 2 --mesh-virtual --rounds 6 --warmup 2 > $O/lenet_mesh2.log 2>&1
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --gpus 2 --mesh-virtual --rounds 6 --warmup 2 > $O/lenet_ring_mesh2.log 2>&1
timeout -k 10 400 python benchmarks/bench_cnn.py --model resnet18 --gpus 2 --mesh-virtual --rounds 2 --warmup 1 > $O/resnet_mesh2.log 2>&1
