#!/bin/bash
# round 4, call O: conflict-free patch swizzle (row & 6) in the layer-1 halo convs: CNN tests, PMC of the
# halo kernels, ResNet-18 A/B against the old swizzle
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-200; case $rc in 0) ;; *) exit $rc;; esac; }
run test_cnn 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cnn_engine_gpu.py
OUT=r4o_pmc bash scripts/gpu_run.sh cnn_pmc || exit 1
python scripts/tools/pmc_table.py $(find gpurun_out/r4o_pmc/cnn_pmc_a -name '*counter_collection.csv' | head -1) $(find gpurun_out/r4o_pmc/cnn_pmc_b -name '*counter_collection.csv' | head -1) > gpurun_out/r4o_pmc/pmc_table.md && grep -E "halo" gpurun_out/r4o_pmc/pmc_table.md
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
run rn_new_a 300 $R
MYFYP_NATIVE_LIB=build/ab_HALO_SWZP0/libmyfyp_hip.so run rn_old_a 300 $R
run rn_new_b 300 $R
MYFYP_NATIVE_LIB=build/ab_HALO_SWZP0/libmyfyp_hip.so run rn_old_b 300 $R
