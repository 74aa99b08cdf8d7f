#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/probes/conv_ab.py > gpurun_out/conv_ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/conv_ab.log | tail -20; exit $rc
