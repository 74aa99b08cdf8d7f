#!/bin/bash
# round 4, call B: fp32 gang layout 2 (owners only, two hand-offs per step): f32 tests (both
# layouts vs torch), headline bench A/B layout 1 vs 2 (alternating), config-5 engine-vs-torch test
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log | cut -c1-400; case $rc in 0) ;; *) exit $rc;; esac; }
run f32_tests 600 python -u -m pytest tests/test_mlp_f32_gpu.py -x -v --timeout 200 --timeout-method thread
for i in 1 2; do
  MYFYP_F32_VARIANT=1 run bench_v1_$i 200 python bench.py --steps 200 --warmup 10
  MYFYP_F32_VARIANT=2 run bench_v2_$i 200 python bench.py --steps 200 --warmup 10
done
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run config5_test 600 python -u -m pytest tests/test_config5_gpu.py -x -v -s --timeout 500 --timeout-method thread
