#!/bin/bash
# experiment: hand-off payloads stored plain (kept in the gang's XCD L2) vs write-through (sc1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_plain; mkdir -p $O
PL=build/plain_PERSIST_PLAIN_PUB1/libmyfyp_hip.so
MYFYP_NATIVE_LIB=$PL timeout -k 10 400 python -u -m pytest tests/test_mlp_f32_gpu.py -q -k "not ks2" --timeout 120 --timeout-method thread > $O/tests_plain.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -1 $O/tests_plain.log
for v in stamps stamps_PERSIST_PLAIN_PUB1; do
  PEERS=8 MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_f32.py > $O/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -E "median" $O/$v.log; [ $rc -eq 0 ] || exit $rc
done
for k in a b; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_base_$k.log 2>&1; rc=$?; echo "== base_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_base_$k.log)"; [ $rc -eq 0 ] || exit $rc
  MYFYP_NATIVE_LIB=$PL timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_plain_$k.log 2>&1; rc=$?; echo "== plain_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_plain_$k.log)"; [ $rc -eq 0 ] || exit $rc
done
