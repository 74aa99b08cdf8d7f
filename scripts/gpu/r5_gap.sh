#!/bin/bash
# stream-operation cost model (scripts/probes/gap_probe.hip), plus its kernel trace
set -o pipefail
O=gpurun_out/r5_gap; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 ./build/gap_probe > $O/gap.log 2>&1 && cat $O/gap.log && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- ./build/gap_probe > $O/gap_prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/prof -name '*.db' | head -1)
python - "$D" > $O/durations.txt <<'PY'
import sqlite3, sys, statistics
from collections import defaultdict
db = sqlite3.connect(sys.argv[1])
rows = list(db.execute("select k.start, k.end, s.kernel_name, k.grid_size_x from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s on k.kernel_id = s.id order by k.start"))
d = defaultdict(list)
for a, b, n, gx in rows:
    d[(n.split("(")[0], gx)].append((b - a) / 1e3)
for (n, gx), v in sorted(d.items()):
    print(f"{n[:60]:60s} grid {gx:7d} n {len(v):4d} median {statistics.median(v):7.2f} us")
PY
cat $O/durations.txt
rm -f "$D"
