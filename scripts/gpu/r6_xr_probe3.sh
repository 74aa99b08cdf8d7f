set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_probe3; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py fedprox,fedprox0,scaffold,scaffold0 2,4 > $O/a.log 2>&1 || exit 1
grep errs $O/*.log
