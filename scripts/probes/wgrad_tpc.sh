set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/w1
for t in ${TPCS:-2 4 8}; do
  MYFYP_WGRAD_TPC=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/w1/t$t -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 1 --n-train 16384 --n-test 2048 > gpurun_out/w1/t$t.log 2>&1 || exit $?
  echo "tpc $t done"
done
