#!/bin/bash
# round 3, call L: the whole GPU suite + smoke on the current tree
set -o pipefail
O=gpurun_out/r3x_l; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "tests rc=$?" >> $O/status
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/status
