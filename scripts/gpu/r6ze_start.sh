# Node-start breakdown of the headline on the late round-6 tree (MYFYP_TIME_PREPARE=1), 3 runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ze_start; mkdir -p $O
for i in 1 2 3; do
  MYFYP_TIME_PREPARE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench_$i.log 2>&1 || exit 1
done
grep -h "prepare\]" $O/bench_1.log | head -20
for f in $O/bench_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['time_to_target_s'], d['node_start_s'], d['time_to_target_from_start_learning_s'])"); done
