#!/bin/bash
# PMC counters for the fused engine kernels (separate run: --pmc only with kernel-trace/stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "mlp_" --output-format csv -d gpurun_out/pmc/a -o a -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc/a.log 2>&1 || { echo "pmc a failed"; tail -20 gpurun_out/pmc/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "mlp_" --output-format csv -d gpurun_out/pmc/b -o b -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc/b.log 2>&1 || { echo "pmc b failed"; tail -20 gpurun_out/pmc/b.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head
