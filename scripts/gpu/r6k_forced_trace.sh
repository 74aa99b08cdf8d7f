# Kernel traces of the one-peer load, plain vs through the RCCL weights plane (--force-collective):
# where the forced path's slow rounds lose their time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6k_forced_trace; mkdir -p $O
for m in plain forced; do
  F=""; [ $m = forced ] && F="--force-collective"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_$m -o run -- python bench.py --peers 1 --n-train 7500 --n-test 1250 --steps 60 --warmup 5 $F > $O/tl_$m.log 2>&1 || exit 1
  D=$(find $O/tl_$m -name '*.db' | head -1)
  python scripts/probes/rocpd_periods.py "$D" mlp_eval_f32 > $O/periods_$m.txt || exit 1
  rm -f "$D"
  head -1 $O/periods_$m.txt
done
