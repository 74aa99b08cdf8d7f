set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probes/start_sampler.py > gpurun_out/sampler.log 2>/dev/null
