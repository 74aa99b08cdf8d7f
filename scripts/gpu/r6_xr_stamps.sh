# Phase stamps of the fp32 epoch at 1 / 2 / 8 peers and owner K splits 1 / 2 / 4 / 8, plus the
# one-peer bench at K splits 2 and 4 (the per-GPU load of the N = 8 run).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_xr_stamps; mkdir -p $O
export MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so
for cfg in "1 8" "1 4" "1 2" "1 1" "2 4" "8 1"; do
  set -- $cfg
  PEERS=$1 MYFYP_F32_KS=$2 timeout -k 10 120 python -u scripts/probes/stamps_f32.py > $O/stamps_p$1_ks$2.log 2>&1 || exit 1
done
unset MYFYP_NATIVE_LIB
for K in 2 4; do
  MYFYP_F32_KS=$K timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --steps 200 --warmup 10 > $O/bench_p1_ks$K.log 2>&1 || exit 1
done
grep -h "median\|peers" $O/stamps_*.log; for f in $O/bench_*.log; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"); done
