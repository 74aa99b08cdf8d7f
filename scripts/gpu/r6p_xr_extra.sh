# XR + extra-term drift: per-parameter errors vs torch, K split 2 / 4 / 8, extras on / off, and the
# discriminating variants (write-through hand-offs, one peer, no momentum).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6p_xr_extra; mkdir -p $O
export MYFYP_F32_XR_EXTRA=1
timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 2,4,8 > $O/a_default.log 2>&1 || exit 1
MYFYP_F32_PLAIN_PUB=0 timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 4 > $O/b_writethrough.log 2>&1 || exit 1
PEERS=1 timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 4,8 > $O/c_p1.log 2>&1 || exit 1
MOM=0 timeout -k 10 200 python -u scripts/probes/xr_extra_probe3.py 4 > $O/d_nomom.log 2>&1 || exit 1
grep -h "ks=" $O/*.log
