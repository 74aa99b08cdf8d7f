#!/bin/bash
# end-of-round-5 numbers for BASELINE configs 3-5 and the 2-member virtual mesh (the N > 1 path on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_configs; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(grep -o '"value": [0-9.]*' $O/$n.log) $(grep -o '"rounds_to_target": [0-9a-z]*' $O/$n.log)"; [ $rc -eq 0 ] || exit $rc; }
run lenet_ring 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3
run resnet_a 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1
run resnet_b 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1
run config5 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 16 --warmup 1 --aggregator fedprox --dirichlet 0.5 --dropout
run mlp_mesh2_virtual 300 python bench.py --gpus 2 --mesh-virtual --steps 100 --warmup 5
