# The one-peer load through the RCCL weights plane (--force-collective: the per-process path of an
# N = 8 torchrun job) with the deferred confirmation lagging one section (default) vs blocking
# (MYFYP_CONFIRM_LAG=0), arms alternating; then the GPU tests of the multi-rank / forced paths.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6j_confirm_lag; mkdir -p $O
b() { timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 --force-collective; }
for i in 1 2; do
  MYFYP_CONFIRM_LAG=0 b > $O/block_$i.log 2>&1 || exit 1
  b > $O/lag_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
grep -h "round-end interval" $O/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "forced or rank or overlap or collective or federation" > $O/tests.log 2>&1 || exit 1
tail -3 $O/tests.log
