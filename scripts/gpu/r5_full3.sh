set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_full3; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1
timeout -k 10 200 python bench.py > $O/bench_default.log 2>&1
bash scripts/gpu/r5_edges.sh > $O/edges.log 2>&1
