# Round 6: cross-XCD K split (XR) of the fp32 epoch — correctness (f32 kernel tests), then the
# per-GPU loads of the N = 8 / 4 / 2 runs (1 / 2 / 4 peers) with and without it, the headline, and
# the mesh GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mlp_f32_gpu.py -x -v --timeout 200 --timeout-method thread > $O/f32_tests.log 2>&1 || exit 1
for P in 1 2 4; do
  N=$((7500 * P))
  timeout -k 10 200 python bench.py --peers $P --n-train $N --steps 200 --warmup 10 > $O/bench_p${P}_xr.log 2>&1 || exit 1
  MYFYP_F32_XSPLIT=0 timeout -k 10 200 python bench.py --peers $P --n-train $N --steps 200 --warmup 10 > $O/bench_p${P}_ks1.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_device_mesh_gpu.py -x -v --timeout 200 --timeout-method thread > $O/mesh_gpu.log 2>&1 || exit 1
tail -2 $O/f32_tests.log; for f in $O/bench_*.log; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['time_to_target_s'])"); done; tail -2 $O/mesh_gpu.log
