#!/bin/bash
# round 4, call I: tuner-free ResNet-18 (config 4) kernel profile: kernel trace over 6 rounds, stats over
# the second half of the optimizer steps (the tuner and the warm-up round are before the window)
set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 5 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; tail -3 $O/prof.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/tools/rocpd_window_stats.py "$T" k_opt_step 0 > $O/resnet_window_stats.csv 2> $O/window.txt && cat $O/window.txt && head -25 $O/resnet_window_stats.csv | cut -c1-200
rm -f "$T"
# headline round timeline with the gather ahead of the epoch (MYFYP_PREP_GATHER=2) vs in the graph
for m in 0 2; do
  MYFYP_PREP_GATHER=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl$m -o run -- python bench.py --steps 40 --warmup 5 > $O/tl$m.log 2>&1
  rc=$?; echo "== tl$m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  D=$(find $O/tl$m -name '*.db' | head -1)
  python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline_prep$m.txt && head -12 $O/timeline_prep$m.txt
  rm -f "$D"
done
