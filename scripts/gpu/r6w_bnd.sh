# Kernel trace of the 8-peer headline: the round boundary (what runs between two epochs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6w_bnd; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python bench.py --steps 40 --warmup 10 > $O/bench.log 2>&1
