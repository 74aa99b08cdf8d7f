set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/start_trace -o run -- python scripts/probes/start_breakdown.py > gpurun_out/start_trace.log 2>&1
