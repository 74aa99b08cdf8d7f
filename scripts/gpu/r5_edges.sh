#!/bin/bash
# device idle at the edges of the 20-round timed window (roctx marks + kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_edges; mkdir -p $O
MYFYP_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1
rc=$?; echo "== trace rc=$rc $(grep -o '"value": [0-9.]*' $O/b.log)"; [ $rc -eq 0 ] || exit $rc
python scripts/probes/window_edges.py $O/tr | tee $O/edges.txt
find $O/tr -name '*.csv' -size +2M -delete
