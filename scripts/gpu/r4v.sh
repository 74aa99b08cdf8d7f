#!/bin/bash
# round 4, call V: where the fused BN finalize tail's time goes (scripts/probes/fin_tail_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export PYTHONPATH=$PWD
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 300 python scripts/probes/fin_tail_probe.py $O/fin_tail.json > $O/probe.log 2>&1; rc=$?; echo "== probe rc=$rc"; cat $O/probe.log | tail -8
