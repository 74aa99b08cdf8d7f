#!/bin/bash
# PMC counters for the CNN engine kernels (each counter set in its own kernel-trace-only run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_cnn; mkdir -p $O
timeout -k 10 120 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || echo "list-avail rc=$?"
want() { for c in "$@"; do grep -q -w "$c" $O/list_avail.txt && printf "%s " "$c"; done; }
BENCH="benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 0 --n-train 4096 --n-test 512"
i=0
for set in \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  cs=$(want $set)
  [ -z "$cs" ] && { echo "set $i: none available"; continue; }
  echo "set $i: $cs"
  timeout -k 10 400 rocprofv3 --pmc $cs --kernel-include-regex "k_conv|k_opt|k_bn" --output-format csv -d $O/s$i -o s -- python3 $BENCH > $O/s$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
find $O -name "*counter_collection*" | head
