#!/bin/bash
# bf16-operand persistent epoch with single-XCD hand-offs: kernel tests + bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_bf16; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "== kernel tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
for k in a b; do
  for v in 1 0; do
    MYFYP_F32_PLAIN_PUB=$v timeout -k 10 200 python bench.py --precision bf16 --steps 200 --warmup 10 > $O/b_p${v}_$k.log 2>&1; rc=$?
    echo "== bf16 plain=$v ($k) rc=$rc $(grep -o '"value": [0-9.]*' $O/b_p${v}_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
