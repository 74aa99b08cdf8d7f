# Headline MLP: the 8-peer one-GPU number, and the per-GPU load of the N = 2 / 4 / 8 runs with the
# test split they actually get (10k / N test images per GPU: each peer evaluates its own partition).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6h_mlp_loads; mkdir -p $O
b() { timeout -k 10 200 python bench.py "$@"; }
b --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
b --steps 200 --warmup 10 > $O/bench200.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 > $O/p1.log 2>&1 || exit 1
b --peers 2 --n-train 15000 --n-test 2500 --steps 200 --warmup 10 > $O/p2.log 2>&1 || exit 1
b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 > $O/p4.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 --force-collective > $O/p1_forced.log 2>&1 || exit 1
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["engine"])')"; done
