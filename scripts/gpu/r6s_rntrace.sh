set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6s_rntrace; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python benchmarks/bench_cnn.py --model resnet18 --rounds 2 --warmup 1 > $O/rn.log 2>&1
ls -laR $O > $O/ls.txt
