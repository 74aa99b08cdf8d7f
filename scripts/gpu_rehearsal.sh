#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 and 4 ranks (gloo weights plane; RCCL refuses two ranks per
# device) through the same bench entry point the driver uses for the scaling runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-rehearsal}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for n in 2 4; do
  MYFYP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2970$n bench.py --gpus $n --steps 10 --warmup 2 > $O/rehearsal_gloo_n$n.log 2>&1
  rc=$?; stop_if_fatal $rc "rehearsal $n"; [ $rc -ne 0 ] && { echo "rehearsal $n failed"; tail -30 $O/rehearsal_gloo_n$n.log; exit 1; }
  echo "n=$n: $(grep '"value"' $O/rehearsal_gloo_n$n.log | cut -c90-220)"
  grep "median ms" $O/rehearsal_gloo_n$n.log | cut -c1-300
done
