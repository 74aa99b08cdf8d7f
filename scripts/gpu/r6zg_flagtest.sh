# The sparse flag-zeroing test on the default build, then its negative control: a build whose
# upload leaves the per-line flags unzeroed must FAIL the same test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zg_flagtest; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py -k "sparse_zeroing or w2_replica or giveup" > $O/default.log 2>&1 || exit 1
tail -n 3 $O/default.log
MYFYP_NATIVE_LIB=build/ab_ENGINE_FLAGS_BROKEN_TEST1/libmyfyp_hip.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py -k "sparse_zeroing" > $O/broken_control.log 2>&1
rc=$?
echo "negative control rc=$rc (1 = the test failed, as it must)"; tail -n 4 $O/broken_control.log
[ $rc -eq 1 ]
