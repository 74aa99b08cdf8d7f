set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_ahead; mkdir -p $O
for i in a b c; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1; done
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b200.log 2>&1
timeout -k 10 700 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_collective_gpu.py tests/test_kernels_gpu.py tests/test_device_mesh_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gpu_mlp.log 2>&1
