#!/bin/bash
# Per-GPU work at N = 1/2/4/8 (8/N peers on one GPU), a multi-rank rehearsal on one GPU (gloo
# weights plane; RCCL refuses two ranks on a device) and a kernel trace of the lone-peer step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-scaling}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for p in 8 4 2 1; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 3 --peers $p > $O/bench_peers$p.log 2>&1
  rc=$?; stop_if_fatal $rc "peers $p"; [ $rc -ne 0 ] && { echo "peers $p failed"; tail -20 $O/bench_peers$p.log; exit 1; }
  echo "peers=$p $(tail -1 $O/bench_peers$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for n in 2 4; do
  MYFYP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2960$n bench.py --gpus $n --steps 10 --warmup 2 > $O/rehearsal_gloo_n$n.log 2>&1
  rc=$?; stop_if_fatal $rc "rehearsal $n"; [ $rc -ne 0 ] && { echo "rehearsal $n failed"; tail -30 $O/rehearsal_gloo_n$n.log; exit 1; }
  echo "rehearsal n=$n: $(tail -1 $O/rehearsal_gloo_n$n.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 bench.py --steps 10 --warmup 2 --peers 1 > $O/prof1.log 2>&1
rc=$?; stop_if_fatal $rc prof1
find $O/prof1 -name "*stats*"
