# Round-6 verification on one MI355X: the whole GPU suite, smoke(), the headline bench (the driver's
# shape), the per-GPU loads of the N = 8 / 4 runs, ResNet-18 config 4, and a kernel-stats profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_verify; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 > $O/p1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --peers 2 --n-train 15000 --n-test 2500 --steps 200 --warmup 10 > $O/p2.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/resnet.log 2>&1 || exit 1
for f in $O/bench20.log $O/p1.log $O/p2.log $O/resnet.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \; ; find $O/prof -name '*.db' -delete; ls $O
