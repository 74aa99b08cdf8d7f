#!/bin/bash
# GPU suite + headline bench (8 peers and 1 peer per GPU) + kernel stats; 8-rank gloo control-plane microbench (CPU only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r1c
O=gpurun_out/r1c
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -m pytest tests -x -q -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; stop_if_fatal $rc pytest
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $O/bench8.log 2>&1 || { echo "bench failed"; tail -30 $O/bench8.log; exit 1; }
tail -1 $O/bench8.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --peers 1 > $O/bench_1peer.log 2>&1 || { echo "bench 1 peer failed"; tail -30 $O/bench_1peer.log; exit 1; }
tail -1 $O/bench_1peer.log; grep '^\[bench\]' $O/bench_1peer.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*stats*"
CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= timeout -k 10 120 python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29623 scripts/probes/gloo_collective_latency.py > $O/gloo8.log 2>&1; grep ms $O/gloo8.log
