set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_async; mkdir -p $O
MYFYP_TIME_PREPARE=1 timeout -k 10 200 python scripts/probes/start_breakdown.py > $O/start.log 2>&1
for i in a b c; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1; done
timeout -k 10 600 python -u -m pytest tests/test_mlp_f32_gpu.py tests/test_collective_gpu.py tests/test_device_mesh_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1
