#!/bin/bash
# round 4 final verification, part 1: the whole GPU test suite and smoke() on the committed tree
set -o pipefail
O=${OUT:-gpurun_out/r4z}; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "== gpu_tests rc=$rc"; tail -5 $O/gpu_tests.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -2 $O/smoke.log; exit $rc
