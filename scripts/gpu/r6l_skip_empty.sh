# Epoch launches only for groups with an active peer: fp32 epoch tests, then the per-GPU loads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6l_skip_empty; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mlp_f32_gpu.py -x -q --timeout 200 --timeout-method thread > $O/f32_tests.log 2>&1 || exit 1
tail -2 $O/f32_tests.log
b() { timeout -k 10 200 python bench.py "$@"; }
b --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 > $O/p1.log 2>&1 || exit 1
b --peers 2 --n-train 15000 --n-test 2500 --steps 200 --warmup 10 > $O/p2.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 --force-collective > $O/p1_forced.log 2>&1 || exit 1
for f in $O/*.log; do case $f in *tests*) continue;; esac; echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
