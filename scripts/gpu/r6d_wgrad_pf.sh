set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6d_wgrad; mkdir -p $O
timeout -k 10 300 python -u scripts/probes/wgrad_pf_ab.py > $O/pf_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "interrupt or prefetch" > $O/tests.log 2>&1 || exit 1
cat $O/pf_ab.log; tail -3 $O/tests.log
