set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s5a.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s5b.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_s5c.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_collective_gpu.py tests/test_device_mesh_gpu.py tests/test_config5_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_sub.log 2>&1
