# Run-time knobs re-checked on the faster late-round-6 epoch (no rebuild): the overlapped
# evaluation's grid cap (MYFYP_EVAL_WGS 16 / 32 default / 64), the prep-stream gather's workgroups
# (MYFYP_PREP_GATHER_WGS 16 / 64 default / 128), and the epoch through its captured graph (MYFYP_EPOCH_GRAPH=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zc_knobs; mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/bench_${tag}.log 2>&1 || exit 1; }
for i in 1 2; do
  run base_$i MYFYP_NOOP=1
  run eval16_$i MYFYP_EVAL_WGS=16
  run eval64_$i MYFYP_EVAL_WGS=64
  run gwgs16_$i MYFYP_PREP_GATHER_WGS=16
  run gwgs128_$i MYFYP_PREP_GATHER_WGS=128
  run graph_$i MYFYP_EPOCH_GRAPH=1
done
for f in $O/bench_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"); done
