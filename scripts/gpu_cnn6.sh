#!/bin/bash
# CNN kernels quick loop: CNN GPU numerics, ResNet-18 bench, kernel stats, VALU/MFMA counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cnn6; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k cnn > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 600 python benchmarks/bench_cnn.py --model resnet18 --rounds 2 > $O/resnet.log 2>&1 || { echo "bench failed"; tail -30 $O/resnet.log; exit 1; }
grep -v amdgpu.ids $O/resnet.log | tail -1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --n-train 8192 --n-test 1024 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "k_conv" --output-format csv -d $O/pmc -o s -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 0 --n-train 4096 --n-test 512 > $O/pmc.log 2>&1 || echo "pmc rc=$?"
python3 scripts/probes/pmc_summary.py $O/pmc/s_counter_collection.csv | cut -c1-200
