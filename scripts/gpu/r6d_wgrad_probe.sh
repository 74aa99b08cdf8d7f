set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6d_wgrad; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/wgrad_atomic_share.py > $O/atomic_share.log 2>&1 || exit 1
cat $O/atomic_share.log
