# The driver's exact headline command, five times on one box: the spread to expect of BENCH_r06.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zj_driver_shape; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/run_$i.log 2>&1 || exit 1
done
for f in $O/run_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['time_to_target_s'], d['final_test_acc'])"); done
