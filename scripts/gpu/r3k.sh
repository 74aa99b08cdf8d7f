#!/bin/bash
# round 3, call K: plain-bench kernel + HIP runtime trace to attribute the per-round blit kernels;
# spill-free build sanity (fp32 MLP tests) and bench
set -o pipefail
O=gpurun_out/r3x_k; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 240 --timeout-method thread > $O/mlp_f32_tests.log 2>&1 || { echo "mlp tests failed" >> $O/status; exit 1; }
for i in 1 2; do timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_$i.log 2>&1 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $O/prof -o run -- python bench.py --steps 40 --warmup 5 > $O/prof.log 2>&1 || { echo "prof rc=$?" >> $O/status; exit 1; }
DB=$(find $O/prof -name '*.db' | head -n 1)
python scripts/probes/rocpd_attrib.py "$DB" > $O/attrib.txt 2>&1
python scripts/probes/rocpd_summary.py "$DB" $O/kernel_stats.csv > $O/summary.txt 2>&1
echo done >> $O/status
