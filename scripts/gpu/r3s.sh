#!/bin/bash
# round 3, call S: fp32 MLP epoch under other scheduler settings (latency bias 0, max-ilp): bench A/B
set -o pipefail
O=gpurun_out/r3x_s; mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for v in main bias0_amdgpuschedulemetricbias0 ilp_amdgpuschedstrategymaxilp; do
    L=build/$v/libmyfyp_hip.so; [ $v = main ] && L=myfyp_amd/_native/libmyfyp_hip.so
    MYFYP_NATIVE_LIB=$L timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$i.log 2>&1 || exit 1
  done
done
echo done >> $O/status
