#!/bin/bash
# GPU check of the CNN engine: kernel numerics + train-step equivalence tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_cnn_engine_gpu.py -x -q -m gpu > gpurun_out/cnn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/cnn_tests.log; tail -40 gpurun_out/cnn_tests.log; exit $rc
