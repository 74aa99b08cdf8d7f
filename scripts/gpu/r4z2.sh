#!/bin/bash
# round 4 final verification, part 2: headline bench and BASELINE configs 3-5 on the committed tree
set -o pipefail
O=${OUT:-gpurun_out/r4z}; mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-400; case $rc in 0) ;; *) exit $rc;; esac; }
run bench_fp32_a 200 python bench.py
run bench_fp32_b 200 python bench.py --steps 200 --warmup 10
run resnet_fedavg 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1
run lenet_ring 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 --warmup 3
run resnet_fedprox_drop 500 python benchmarks/bench_cnn.py --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 16 --warmup 1
