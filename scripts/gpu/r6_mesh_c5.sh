# Round 6: mesh guard / mesh aggregator GPU tests, then the config-5 calibration for fixed bounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_mesh_c5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_device_mesh_gpu.py -x -v --timeout 200 --timeout-method thread > $O/mesh_gpu.log 2>&1 || exit 1
timeout -k 10 700 python -u scripts/probes/config5_calibrate2.py e1 e2 e3 t1 t2 t3 > $O/c5_clean.log 2>&1 || exit 1
MYFYP_DEBUG_LR_SCALE=1.05 timeout -k 10 300 python -u scripts/probes/config5_calibrate2.py e1 e2 > $O/c5_mut.log 2>&1 || exit 1
tail -3 $O/mesh_gpu.log; grep scale= $O/c5_clean.log $O/c5_mut.log
