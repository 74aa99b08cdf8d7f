# Last check of the committed end-of-round tree: GPU suite, smoke(), the driver-shaped headline and
# a 200-round headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_final3; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -n 2 $O/gpu_suite.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench200.log 2>&1 || exit 1
for f in $O/bench20.log $O/bench200.log; do echo "$f $(tail -n 1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["time_to_target_s"], d["final_test_acc"], d["config"]["engine"])')"; done
