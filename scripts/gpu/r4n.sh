#!/bin/bash
# round 4, call N: stride-2 dgrad — parity-class DMA path (MYFYP_CNN_S2_FWD=1) vs the register-staged
# k_conv_gemm<2>: PMC tables (VALU/MFMA, wait share) and ResNet-18 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=r4n_pmc_base bash scripts/gpu_run.sh cnn_pmc || exit 1
MYFYP_CNN_S2_FWD=1 OUT=r4n_pmc_s2 bash scripts/gpu_run.sh cnn_pmc || exit 1
for d in r4n_pmc_base r4n_pmc_s2; do
  python scripts/tools/pmc_table.py $(find gpurun_out/$d/cnn_pmc_a -name '*counter_collection.csv' | head -1) $(find gpurun_out/$d/cnn_pmc_b -name '*counter_collection.csv' | head -1) > gpurun_out/$d/pmc_table.md && grep -E "k_conv_gemm<2|k_conv_fwd_dma<5|halo<4" gpurun_out/$d/pmc_table.md
done
O=gpurun_out/r4n; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-200; case $rc in 0) ;; *) exit $rc;; esac; }
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
run rn_base_a 300 $R
MYFYP_CNN_S2_FWD=1 run rn_s2_a 300 $R
run rn_base_b 300 $R
MYFYP_CNN_S2_FWD=1 run rn_s2_b 300 $R
