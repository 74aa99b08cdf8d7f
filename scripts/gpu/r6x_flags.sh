# Flag-block zeroing between epochs: one store per flag line (default) vs every word (before),
# fp32 / kernel tests on the default, then alternating 200-round benches + a boundary trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6x_flags; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in base ab_ENGINE_FLAGS_DENSE1; do
    if [ $v = base ]; then unset MYFYP_NATIVE_LIB; else export MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 --peers 1 --n-train 7500 --n-test 1250 > $O/bench_p1_${v}_$i.log 2>&1 || exit 1
  done
done
unset MYFYP_NATIVE_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python bench.py --steps 40 --warmup 10 > $O/trace_bench.log 2>&1 || exit 1
for f in $O/bench_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"); done
