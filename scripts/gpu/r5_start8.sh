set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in a b c; do timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_s8$i.log 2>&1; done
for i in d e; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s8$i.log 2>&1; done
