# cProfile of the 8 Node.start() calls of the headline (node start is about half of time-to-target).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zf_startprof; mkdir -p $O
MYFYP_PROFILE_START=$O/start.prof timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit 1
python - <<'PY' > $O/pstats.txt
import pstats
s = pstats.Stats("gpurun_out/r6zf_startprof/start.prof"); s.sort_stats("cumulative").print_stats(60); s.sort_stats("tottime").print_stats(30)
PY
tail -n 1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['time_to_target_s'], d['node_start_s'])"
