#!/bin/bash
# round 4, call P: direct-X fp32 epochs (layout 1 reads batch rows from a static bf16 copy through the
# epoch index; no per-epoch image gather): MLP GPU tests, stamps, timeline, bench A/B vs the gathered build
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log | cut -c1-260; case $rc in 0) ;; *) exit $rc;; esac; }
run test_mlp 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py tests/test_collective_gpu.py
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so run stamps_v1 200 python scripts/probes/stamps_f32.py
run bench_xd_a 200 python bench.py --steps 200 --warmup 10
MYFYP_NATIVE_LIB=build/ab_P32_XDIRECT0/libmyfyp_hip.so run bench_gath_a 200 python bench.py --steps 200 --warmup 10
run bench_xd_b 200 python bench.py --steps 200 --warmup 10
MYFYP_NATIVE_LIB=build/ab_P32_XDIRECT0/libmyfyp_hip.so run bench_gath_b 200 python bench.py --steps 200 --warmup 10
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run -- python bench.py --steps 40 --warmup 5 > $O/tl.log 2>&1
rc=$?; echo "== tl rc=$rc"; [ $rc -eq 0 ] || exit $rc
D=$(find $O/tl -name '*.db' | head -1)
python scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline.txt && cut -c1-120 $O/timeline.txt | tail -12
rm -f "$D"
