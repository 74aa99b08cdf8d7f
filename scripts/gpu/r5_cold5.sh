set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MYFYP_TIME_PREPARE=1 timeout -k 10 200 python scripts/probes/start_breakdown.py > gpurun_out/start_h.log 2>&1
for i in a b; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s11$i.log 2>&1; done
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_s11c.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_collective_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_mlp2.log 2>&1
