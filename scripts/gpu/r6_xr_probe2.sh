set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_probe2; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py fedprox,fedprox,sgdm,adam,sgdm 4 > $O/a_p2.log 2>&1 || exit 1
PEERS=1 timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py sgdm,sgdm,adam,fedprox 8 > $O/b_p1.log 2>&1 || exit 1
PEERS=1 MYFYP_PREP_GATHER=0 timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py sgdm,sgdm,adam 8 > $O/c_p1_nogather.log 2>&1 || exit 1
PEERS=1 timeout -k 10 300 python -u scripts/probes/xr_extra_probe.py sgdm,adam 1,2 > $O/d_p1_ks12.log 2>&1 || exit 1
grep errs $O/*.log
