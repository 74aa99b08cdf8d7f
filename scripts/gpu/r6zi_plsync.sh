# A/B: heads hand the H2 tile to the partial logits through a wave-local LDS fence instead of a
# workgroup barrier (P32_PL_WAVESYNC). fp32 tests on the variant, stamps, alternated benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zi_plsync; mkdir -p $O
MYFYP_NATIVE_LIB=build/ab_P32_PL_WAVESYNC1/libmyfyp_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py > $O/tests.log 2>&1 || exit 1
for v in stamps stamps_P32_PL_WAVESYNC1; do
  MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so PEERS=8 MYFYP_F32_KS=1 timeout -k 10 120 python -u scripts/probes/stamps_f32.py > $O/stamps_$v.log 2>&1 || exit 1
done
for i in 1 2 3; do
  for v in base ab_P32_PL_WAVESYNC1; do
    if [ $v = base ]; then unset MYFYP_NATIVE_LIB; else export MYFYP_NATIVE_LIB=build/$v/libmyfyp_hip.so; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 --peers 1 --n-train 7500 --n-test 1250 > $O/bench_p1_${v}_$i.log 2>&1 || exit 1
  done
done
unset MYFYP_NATIVE_LIB
grep -h "median\|->" $O/stamps_*.log
for f in $O/bench_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"); done
