#!/bin/bash
# round 4, call M: evaluation-side host wait polled (not hipEventSynchronize); bench A/B + timeline
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -4 $O/$n.log | cut -c1-260; case $rc in 0) ;; *) exit $rc;; esac; }
run bench_a 200 python bench.py --steps 200 --warmup 10
MYFYP_GRAPH_PUBLISH=0 run bench_nogp_a 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=0 run bench_prep0_a 200 python bench.py --steps 200 --warmup 10
run bench_b 200 python bench.py --steps 200 --warmup 10
MYFYP_GRAPH_PUBLISH=0 run bench_nogp_b 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=0 run bench_prep0_b 200 python bench.py --steps 200 --warmup 10
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-120 $O/timeline.txt | tail -12
rm -f "$D"
