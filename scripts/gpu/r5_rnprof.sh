set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_rnprof; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 5 --warmup 1 > $O/rn.log 2>&1
