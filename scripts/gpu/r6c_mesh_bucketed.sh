# Round 6: bucketed / delayed mesh FedAvg on the GPU (RCCL G = 1 and virtual members), then the
# virtual-mesh bench (the mesh path's host cost) with the bucketed exchange as default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c_mesh; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_device_mesh_gpu.py -x -v --timeout 200 --timeout-method thread > $O/mesh_gpu.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --steps 50 --warmup 5 > $O/bench_v8.log 2>&1 || exit 1
tail -3 $O/mesh_gpu.log; tail -1 $O/bench_v8.log
