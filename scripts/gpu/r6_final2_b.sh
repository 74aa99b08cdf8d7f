# Round-6 final verification (after the poll / softmax / flag-zeroing changes), part 2: benches + profile.
# loads of the N = 8 / 4 / 2 runs, configs 3-5, and a kernel-stats profile of the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6_final2; mkdir -p $O
b() { timeout -k 10 200 python bench.py "$@"; }
b --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
b --steps 200 --warmup 10 > $O/bench200.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 > $O/p1.log 2>&1 || exit 1
b --peers 2 --n-train 15000 --n-test 2500 --steps 200 --warmup 10 > $O/p2.log 2>&1 || exit 1
b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 > $O/p4.log 2>&1 || exit 1
b --peers 1 --n-train 7500 --n-test 1250 --steps 200 --warmup 10 --force-collective > $O/p1_forced.log 2>&1 || exit 1
# 4 peers per GPU (N = 2): K split 2 (cross-XCD) against the default K split 1, alternated
MYFYP_F32_KS=2 b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 > $O/p4_ks2.log 2>&1 || exit 1
b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 > $O/p4_b.log 2>&1 || exit 1
MYFYP_F32_KS=2 b --peers 4 --n-train 30000 --n-test 5000 --steps 200 --warmup 10 > $O/p4_ks2_b.log 2>&1 || exit 1
b --gpus 8 --mesh-virtual --steps 50 --warmup 5 > $O/mesh_virtual8.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/resnet.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 > $O/lenet_ring.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 16 > $O/config5.log 2>&1 || exit 1
for f in $O/mesh_virtual8.log $O/bench20.log $O/bench200.log $O/p1.log $O/p2.log $O/p4.log $O/p1_forced.log $O/p4_ks2.log $O/p4_b.log $O/p4_ks2_b.log $O/resnet.log $O/lenet_ring.log $O/config5.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("time_to_target_s"), d.get("final_test_acc", d.get("final_test_acc_mean")))')"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $O/prof.log 2>&1 || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \; ; rm -rf $O/prof; ls $O
