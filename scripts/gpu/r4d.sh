#!/bin/bash
# round 4, call D: layout 2 after moving dW3 to reducer partials (f32 tests, stamps, bench A/B);
# CNN: BN1 folded into the layer-1 patch-staged kernels (kernel test, CNN tests, ResNet A/B)
set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
run f32_tests 600 python -u -m pytest tests/test_mlp_f32_gpu.py -x -v --timeout 200 --timeout-method thread -k "v2 or giveup or eval or partial or prewarm"
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=2 run stamps_v2 200 python scripts/probes/stamps_f32v2.py
for i in 1 2; do
  MYFYP_F32_VARIANT=1 run bench_v1_$i 200 python bench.py --steps 200 --warmup 10
  MYFYP_F32_VARIANT=2 run bench_v2_$i 200 python bench.py --steps 200 --warmup 10
done
run cnn_halo_test 300 python -u -m pytest tests/test_cnn_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "bn_prologue_in_patch or resnet"
for i in 1 2; do
  MYFYP_CNN_HALO_BN1=0 run resnet_nofold_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 6
  run resnet_fold_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 6
done
