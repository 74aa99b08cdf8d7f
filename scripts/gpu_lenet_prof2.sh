#!/bin/bash
# Kernel trace of the config-3 bench (fused LeNet step) for gap / per-kernel analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-lenetprof2}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 3 > $O/lenet_prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 $O/lenet_prof.log; exit $rc; }
grep '"value"' $O/lenet_prof.log | cut -c1-200
head -8 $O/prof/run_kernel_stats.csv | cut -c1-150
