# Prices the work beside the headline epoch: the 8-peer headline with the next
# epoch's gather and / or the overlapped evaluation turned off (debug knobs: data re-read, results
# zero), arms alternating, 200 timed rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6o_interference; mkdir -p $O
b() { timeout -k 10 200 python bench.py --steps 200 --warmup 10; }
for i in 1 2; do
  b > $O/base_$i.log 2>&1 || exit 1
  MYFYP_DEBUG_NO_GATHER=1 b > $O/nogather_$i.log 2>&1 || exit 1
  MYFYP_DEBUG_NO_EVAL=1 b > $O/noeval_$i.log 2>&1 || exit 1
  MYFYP_DEBUG_NO_GATHER=1 MYFYP_DEBUG_NO_EVAL=1 b > $O/none_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
