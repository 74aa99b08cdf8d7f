# The N = 2 per-GPU load (4 peers) at K split 1 (default) vs the cross-XCD K split 2, now that the
# launcher skips empty groups; arms alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6r_p4_ks2; mkdir -p $O
b() { timeout -k 10 200 python bench.py --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10; }
for i in 1 2; do
  b > $O/ks1_$i.log 2>&1 || exit 1
  MYFYP_F32_KS=2 b > $O/ks2_$i.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["final_test_acc"], d["config"]["engine"])')"; done
