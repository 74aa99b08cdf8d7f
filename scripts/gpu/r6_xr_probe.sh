set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_probe; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py fedprox,sgdm,scaffold 1,2,4,8 > $O/probe.log 2>&1 || exit 1
MYFYP_F32_PLAIN_PUB=0 timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py fedprox,sgdm 8 > $O/probe_wt.log 2>&1 || exit 1
PEERS=1 timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py fedprox,sgdm 8 > $O/probe_p1.log 2>&1 || exit 1
grep errs $O/*.log
