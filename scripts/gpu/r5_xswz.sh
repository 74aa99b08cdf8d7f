#!/bin/bash
# swizzled X tile vs the r4 layout
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_xswz; mkdir -p $O
OLD=build/xs_P32_XSWZ0/libmyfyp_hip.so
timeout -k 10 500 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "== tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
for v in new old; do
  L=""; [ $v = old ] && L=$OLD
  MYFYP_NATIVE_LIB=$L timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA \
    --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/p_$v -o p -- python3 bench.py --steps 3 --warmup 2 > $O/p_$v.log 2>&1 || exit 1
  python3 scripts/probes/pmc_summary.py $(find $O/p_$v -name '*counter_collection.csv') > $O/pmc_$v.txt; cat $O/pmc_$v.txt
done
for k in a b c; do
  for v in new old; do
    L=""; [ $v = old ] && L=$OLD
    MYFYP_NATIVE_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_${v}_$k.log 2>&1; rc=$?
    echo "== $v ($k) rc=$rc $(grep -o '"value": [0-9.]*' $O/b_${v}_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
