set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_probe4; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/xr_extra_probe2.py 2,4,8 > $O/a.log 2>&1 || exit 1
grep err $O/a.log
