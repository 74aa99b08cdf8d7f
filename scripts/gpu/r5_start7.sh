set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in a b c; do timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_s7$i.log 2>&1; done
