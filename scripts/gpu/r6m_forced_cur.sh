# Critical-path FedAvg on the compute stream (reduce writes the retained copy): the forced one-peer
# load, the per-GPU loads again, and the GPU tests of the forced / overlap / fault paths.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6m_forced_cur; mkdir -p $O
b() { timeout -k 10 200 python bench.py "$@"; }
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 --force-collective > $O/p1_forced.log 2>&1 || exit 1
b --peers 2 --n-train 15000 --n-test 2500 --steps 200 --warmup 10 --force-collective > $O/p2_forced.log 2>&1 || exit 1
b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 --force-collective > $O/p4_forced.log 2>&1 || exit 1
b --steps 20 --warmup 3 --force-collective > $O/p8_forced.log 2>&1 || exit 1
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "forced or rank or overlap or collective or federation or fault" > $O/tests.log 2>&1 || exit 1
tail -3 $O/tests.log
