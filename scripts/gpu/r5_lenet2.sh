set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_lenet2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cnn_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "lenet" > $O/tests.log 2>&1
for i in a b; do timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3 > $O/lenet_$i.log 2>&1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -- python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 10 --warmup 2 > $O/prof.log 2>&1
