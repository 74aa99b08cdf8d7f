#!/bin/bash
# single-XCD gangs: payloads + flags plain (1) vs payloads only (2) vs write-through (0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_plain3; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 2; do
  MYFYP_F32_PLAIN_PUB=$v PEERS=8 MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_f32.py > $O/stamps_plain$v.log 2>&1
  rc=$?; echo "== stamps plain=$v rc=$rc"; grep -E "median" $O/stamps_plain$v.log; [ $rc -eq 0 ] || exit $rc
done
for k in a b c; do
  for v in 1 2 0; do
    MYFYP_F32_PLAIN_PUB=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_p${v}_$k.log 2>&1; rc=$?; echo "== p${v}_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_p${v}_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
