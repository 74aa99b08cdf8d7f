#!/bin/bash
# round 4, end: ResNet-18 conv / BN / optimizer PMC table on the final tree (two counter passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=r4pmc bash scripts/gpu_run.sh cnn_pmc || exit 1
python scripts/tools/pmc_table.py $(find gpurun_out/r4pmc/cnn_pmc_a -name '*counter_collection.csv' | head -1) $(find gpurun_out/r4pmc/cnn_pmc_b -name '*counter_collection.csv' | head -1) > gpurun_out/r4pmc/pmc_table.md && head -40 gpurun_out/r4pmc/pmc_table.md
find gpurun_out/r4pmc -name '*counter_collection.csv' -delete
