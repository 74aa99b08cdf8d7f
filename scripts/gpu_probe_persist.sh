#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-probe}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python -X faulthandler scripts/probes/stamps_persistent.py > $O/stamps.log 2>&1
rc=$?; cat $O/stamps.log | tail -20; stop_if_fatal $rc stamps
timeout -k 10 240 python scripts/probes/stack_sampler.py --steps 20 --warmup 3 > $O/sampler_persist.log 2>&1
rc=$?; stop_if_fatal $rc samp1
MYFYP_MLP_PERSISTENT=0 timeout -k 10 240 python scripts/probes/stack_sampler.py --steps 20 --warmup 3 > $O/sampler_steps.log 2>&1
rc=$?; stop_if_fatal $rc samp2
grep '"value"' $O/sampler_*.log | cut -c1-200
