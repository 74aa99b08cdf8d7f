#!/bin/bash
# round 4, call G: layout-1 head softmax over 8 waves (P32_SM8): f32 numerics tests, stamps, bench A/B
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -4 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
run test_f32 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so run stamps_v1 200 python scripts/probes/stamps_f32.py
run bench_sm8_a 200 python bench.py --steps 200 --warmup 10
MYFYP_NATIVE_LIB=build/ab_P32_SM80/libmyfyp_hip.so run bench_sm4_a 200 python bench.py --steps 200 --warmup 10
run bench_sm8_b 200 python bench.py --steps 200 --warmup 10
MYFYP_NATIVE_LIB=build/ab_P32_SM80/libmyfyp_hip.so run bench_sm4_b 200 python bench.py --steps 200 --warmup 10
