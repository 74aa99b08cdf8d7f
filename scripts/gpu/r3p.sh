#!/bin/bash
# round 3, call P: kernel trace of the headline bench with the gather on the prep stream
set -o pipefail
O=gpurun_out/r3x_p; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MYFYP_PREP_GATHER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 40 --warmup 5 > $O/prof.log 2>&1 || { echo "prof rc=$?" >> $O/status; exit 1; }
for i in 1 2; do
  MYFYP_PREP_GATHER=1 timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_prep_$i.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_graph_$i.log 2>&1 || exit 1
done
echo done >> $O/status
