#!/bin/bash
# round 3, call J: flag protocol vs LL per hand-off (partial logits only, dH2 only): bench A/B/C twice
set -o pipefail
O=gpurun_out/r3x_j; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 240 --timeout-method thread > $O/mlp_f32_tests.log 2>&1 || { echo "mlp tests failed" >> $O/status; exit 1; }
for i in 1 2; do
  for v in main llpl_P32_LL_PL1 lldh_P32_LL_DH21; do
    L=build/$v/libmyfyp_hip.so; [ $v = main ] && L=myfyp_amd/_native/libmyfyp_hip.so
    MYFYP_NATIVE_LIB=$L timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$i.log 2>&1 || exit 1
  done
done
echo done >> $O/status
# ResNet-18 difficulty calibration (rounds_to_target >= 5, final < 0.99)
for s in 0.85 0.9; do
  timeout -k 10 240 python benchmarks/bench_cnn.py --model resnet18 --rounds 12 --warmup 1 --similarity $s --noise 1.2 --modes 4 --label-noise 0.1 --target-acc 0.9 > $O/resnet_sim$s.log 2>&1 || exit 1
done
echo cnn done >> $O/status
