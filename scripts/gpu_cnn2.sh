#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_cnn_engine_gpu.py -x -q -m gpu > gpurun_out/cnn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cnn_tests.log; [ $rc -eq 0 ] || { grep -B2 -A20 "^E " gpurun_out/cnn_tests.log | head -60; exit $rc; }
timeout -k 10 600 python benchmarks/bench_cnn.py --model resnet18 --rounds 2 --torch-step > gpurun_out/cnn_resnet_fedavg.log 2>&1 || { tail -20 gpurun_out/cnn_resnet_fedavg.log; exit 1; }
tail -1 gpurun_out/cnn_resnet_fedavg.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --n-train 8192 --n-test 1024 > gpurun_out/prof_cnn.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_cnn.log; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_cnn/run_kernel_stats.csv")))
for r in rows[:16]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>6} avg_us={float(r["AverageNs"])/1e3:9.1f} pct={float(r["Percentage"]):6.2f}')
PY
