set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MYFYP_TIME_PREPARE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/start_trace2 -o run -- python scripts/probes/start_breakdown.py > gpurun_out/start_trace2.log 2>&1
MYFYP_TIME_PREPARE=1 timeout -k 10 200 python scripts/probes/start_breakdown.py > gpurun_out/start_d.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s1.log 2>&1
