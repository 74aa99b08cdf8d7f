#!/bin/bash
# ResNet-18: batched weight flips (one launch per backward) vs per-layer; fused BN finalize re-check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_flip; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_cnn_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1
rc=$?; echo "== tests rc=$rc"; tail -1 $O/cnn_tests.log; [ $rc -eq 0 ] || exit $rc
for i in a b c; do
  for v in base noflip fin; do
    case $v in
      base) env=() ;;
      noflip) env=(MYFYP_CNN_FLIP_BATCH=0) ;;
      fin) env=(MYFYP_CNN_FUSE_FIN=1) ;;
    esac
    env "${env[@]}" timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1 > $O/rn_${v}_$i.log 2>&1
    rc=$?; echo "== rn_${v}_$i rc=$rc $(grep -o '"value": [0-9.]*' $O/rn_${v}_$i.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
