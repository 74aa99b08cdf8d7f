#!/bin/bash
# end-of-round kernel statistics of the headline (40 timed rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_final_prof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || exit 1
find $O/p -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/p -name '*kernel_trace.csv' -size +4M -delete
head -12 $O/kernel_stats.csv | cut -c1-200
