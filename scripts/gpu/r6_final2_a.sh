# Round-6 final verification (after the poll / softmax / flag-zeroing changes), part 1: GPU suite + smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_final2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
