set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MYFYP_ROCTX=1 timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/bench_trace4 -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/bench_trace4.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s4a.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s4b.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_s4c.log 2>&1
