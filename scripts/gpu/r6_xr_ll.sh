# XR with dH2 as LL pairs: correctness (XR tests), stamps, and the 1 / 2 peer benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_ll; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mlp_f32_gpu.py -x -v --timeout 200 --timeout-method thread -k "ks4 or ks8 or bit_identical or giveup or w2_replica" > $O/f32_tests.log 2>&1 || exit 1
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so PEERS=1 MYFYP_F32_KS=8 timeout -k 10 120 python -u scripts/probes/stamps_f32.py > $O/stamps_p1_ks8.log 2>&1 || exit 1
for P in 1 2; do
  timeout -k 10 200 python bench.py --peers $P --n-train $((7500 * P)) --steps 200 --warmup 10 > $O/bench_p${P}_xr.log 2>&1 || exit 1
done
tail -1 $O/f32_tests.log; grep -h "median" $O/stamps_*.log; for f in $O/bench_*.log; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['engine'])"); done
timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --force-collective --steps 200 --warmup 10 > $O/bench_p1_forced.log 2>&1 || exit 1
tail -1 $O/bench_p1_forced.log
