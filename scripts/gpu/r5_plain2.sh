#!/bin/bash
# hand-off payloads stored plain when the gang sits on one XCD (run-time check) vs always write-through
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_plain2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MYFYP_F32_PLAIN_PUB=$v PEERS=8 MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_f32.py > $O/stamps_plain$v.log 2>&1
  rc=$?; echo "== stamps plain=$v rc=$rc"; grep -E "median" $O/stamps_plain$v.log; [ $rc -eq 0 ] || exit $rc
done
for k in a b c; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_plain_$k.log 2>&1; rc=$?; echo "== plain_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_plain_$k.log)"; [ $rc -eq 0 ] || exit $rc
  MYFYP_F32_PLAIN_PUB=0 timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_wt_$k.log 2>&1; rc=$?; echo "== wt_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_wt_$k.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1; rc=$?; echo "== bench20 rc=$rc $(grep -o '"value": [0-9.]*' $O/bench20.log) $(grep -o '"time_to_target_s": [0-9.]*' $O/bench20.log)"
