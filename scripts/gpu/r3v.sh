#!/bin/bash
# round 3, call V: where the first rounds' time goes (time-to-accuracy startup)
set -o pipefail
O=gpurun_out/r3x_v; mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2; do timeout -k 10 120 python bench.py --steps 50 --warmup 5 > $O/bench_$i.log 2>&1 || exit 1; done
timeout -k 10 120 python scripts/probes/py_profile_bench.py > $O/pyprof.log 2>&1; echo "pyprof rc=$?" >> $O/status
echo done >> $O/status
