#!/bin/bash
# round 3, call W: engine prewarm at Node.start: tests, bench (time-to-accuracy) with/without
set -o pipefail
O=gpurun_out/r3x_w; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_mlp_f32_gpu.py -x -v --timeout 240 --timeout-method thread -k "prewarm or giveup or epoch_matches" > $O/tests.log 2>&1 || { echo "tests failed" >> $O/status; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_warm_$i.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-prewarm > $O/bench_cold_$i.log 2>&1 || exit 1
done
echo done >> $O/status
