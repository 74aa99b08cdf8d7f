# Round-6 starting point: GPU suite, headline bench, and the one-peer-per-GPU load (the device
# work of one GPU of the N = 8 run) at K split 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_start; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --steps 200 --warmup 10 > $O/bench_p1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --peers 2 --n-train 15000 --steps 200 --warmup 10 > $O/bench_p2.log 2>&1 || exit 1
tail -2 $O/gpu_suite.log; tail -1 $O/bench20.log; tail -1 $O/bench_p1.log; tail -1 $O/bench_p2.log
