#!/bin/bash
# round 3, call M: ResNet-18 (config 4) kernel trace for a per-step breakdown; conv fwd/dgrad per-layer timings
set -o pipefail
O=gpurun_out/r3x_m; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 3 --warmup 1 > $O/prof.log 2>&1 || { echo "prof rc=$?" >> $O/status; exit 1; }
DB=$(find $O/prof -name '*.db' | head -n 1)
python scripts/probes/rocpd_summary.py "$DB" $O/kernel_stats.csv > $O/summary.txt 2>&1
python scripts/probes/rocpd_timeline.py "$DB" k_input_prep > $O/timeline.txt 2>&1
timeout -k 10 120 python scripts/probes/conv_ab.py > $O/conv_ab.log 2>&1
echo done >> $O/status
