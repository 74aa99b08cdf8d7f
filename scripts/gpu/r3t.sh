#!/bin/bash
# round 3, call T: LeNet-5 ring (config 3) kernel trace: per-round device timeline
set -o pipefail
O=gpurun_out/r3x_t; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?" >> $O/status; exit 1; }
DB=$(find $O/prof -name '*.db' | head -n 1)
python scripts/probes/rocpd_summary.py "$DB" $O/kernel_stats.csv > $O/summary.txt 2>&1
timeout -k 10 200 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 > $O/bench.log 2>&1
echo done >> $O/status
