#!/bin/bash
# round 3, call Q: fp32 MLP epoch, scheduling fences between K steps on/off (forward, C2): bench A/B
set -o pipefail
O=gpurun_out/r3x_q; mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in sb00_P32_SB_FWD0_P32_SB_C20; do
  MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed" >> $O/status; exit 1; }
done
for i in 1 2; do
  for v in main sbf0_P32_SB_FWD0 sbc0_P32_SB_C20 sb00_P32_SB_FWD0_P32_SB_C20; do
    L=build/$v/libmyfyp_hip.so; [ $v = main ] && L=myfyp_amd/_native/libmyfyp_hip.so
    MYFYP_NATIVE_LIB=$L timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$i.log 2>&1 || exit 1
  done
done
echo done >> $O/status
