set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_probe5; mkdir -p $O
MYFYP_DEBUG_NO_EXTRA=1 timeout -k 10 300 python -u scripts/probes/xr_extra_probe2.py 4 > $O/a.log 2>&1 || exit 1
MYFYP_F32_PLAIN_PUB=0 timeout -k 10 300 python -u scripts/probes/xr_extra_probe2.py 4 > $O/b.log 2>&1 || exit 1
grep err $O/*.log
