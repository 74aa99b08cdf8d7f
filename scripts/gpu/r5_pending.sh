set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_pending; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
for i in a b; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_$i.log 2>&1; done
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b200.log 2>&1
