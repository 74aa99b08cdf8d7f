set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probes/cold_probe.py > gpurun_out/cold_3.log 2>&1
MYFYP_TIME_PREPARE=1 timeout -k 10 200 python scripts/probes/start_breakdown.py > gpurun_out/start_e.log 2>&1
