#!/bin/bash
# gather ahead ordered after the overlapped evaluation (one event record fewer per round) vs its own event
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_evalorder; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "== tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
for k in a b c; do
  for v in 1 0; do
    MYFYP_EVAL_GATHER_ORDER=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_${v}_$k.log 2>&1; rc=$?
    echo "== order=$v ($k) rc=$rc $(grep -o '"value": [0-9.]*\|"time_to_target_s": [0-9.]*' $O/b_${v}_$k.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1 || exit 1
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-120 $O/timeline.txt | tail -12
rm -f "$D"
