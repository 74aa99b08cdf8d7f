# Round-5 verification: GPU suite, plain bench, virtual 8-member mesh bench (host cost of the mesh
# path on one GPU; not a scaling measurement), CNN config-4 bench.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_n1.log 2>&1
timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --steps 100 --warmup 10 > gpurun_out/bench_virt8.log 2>&1
timeout -k 10 200 python bench.py --gpus 2 --mesh-virtual --steps 100 --warmup 10 > gpurun_out/bench_virt2.log 2>&1
