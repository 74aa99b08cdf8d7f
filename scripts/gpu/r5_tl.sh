#!/bin/bash
# round 5: current headline round boundary (kernel-trace timeline of the main stream)
set -o pipefail
O=gpurun_out/${TL_OUT:-r5_tl}; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-160 $O/timeline.txt | tail -40
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 > $O/timeline_all.txt
rm -f "$D"
