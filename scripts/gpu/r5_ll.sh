#!/bin/bash
# LL (value, tag) hand-offs with plain stores for single-XCD gangs, per hand-off, vs the drained-flag default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_ll; mkdir -p $O
if [ "${SKIP_PRE:-0}" != 1 ]; then
timeout -k 10 500 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_default.log 2>&1
rc=$?; echo "== f32 tests (default lib, layout 2 single-XCD too) rc=$rc $(tail -1 $O/tests_default.log)"; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  MYFYP_F32_VARIANT=2 MYFYP_F32_PLAIN_PUB=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_v2_plain$v.log 2>&1; rc=$?
  echo "== layout 2 plain=$v rc=$rc $(grep -o '"value": [0-9.]*' $O/b_v2_plain$v.log)"; [ $rc -eq 0 ] || exit $rc
done
fi
V="ll_P32_LL_PL1 ll_P32_LL_DH21 ll_P32_LL_H11 ll_P32_LL_PL1_P32_LL_DH21_P32_LL_H11 ab_P32_BALANCE1 ab_P32_SB_FWD0"
for v in $V; do
  MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread -k "matches_torch_adam and v1ks1" > $O/t_$v.log 2>&1
  rc=$?; echo "== test $v rc=$rc $(tail -1 $O/t_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
PEERS=8 MYFYP_NATIVE_LIB=build/stamps_P32_LL_PL1_P32_LL_DH21_P32_LL_H11/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_f32.py > $O/stamps_ll_all.log 2>&1
rc=$?; echo "== stamps rc=$rc"; grep median $O/stamps_ll_all.log; [ $rc -eq 0 ] || exit $rc
for k in a b; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_base_$k.log 2>&1; rc=$?; echo "== base_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/b_base_$k.log)"; [ $rc -eq 0 ] || exit $rc
  for v in $V; do
    MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_${v}_$k.log 2>&1; rc=$?
    echo "== ${v}_$k rc=$rc $(grep -o '"value": [0-9.]*' $O/b_${v}_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
