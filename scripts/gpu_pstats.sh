#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pstats}
mkdir -p $O
PSTATS_OUT=$O/bench.pstats timeout -k 10 300 python scripts/probes/py_profile_bench.py --steps 60 --warmup 3 > $O/pyprof.log 2>&1
rc=$?; grep '"value"' $O/pyprof.log | cut -c90-150; exit $rc
