set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_lenet; mkdir -p $O
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 > $O/lenet.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 10 --warmup 2 > $O/lenet_prof.log 2>&1
