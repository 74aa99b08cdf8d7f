#!/bin/bash
# round 4, call A: config-5 bisect (15 rounds each, same seeds) + headline bench on a fresh box
#  a: Dirichlet(0.5) + FedProx + dropout (config 5 as is)   b: IID + FedProx
#  c: Dirichlet(0.5) + FedAvg, no dropout                   d: (a) on the torch autograd learner
#  e: Dirichlet(0.5) + FedProx, no dropout
set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-600; case $rc in 0) ;; *) exit $rc;; esac; }
run bench 200 python bench.py
R="benchmarks/bench_cnn.py --model resnet18 --rounds 15 --warmup 1"
run c5_a 300 python $R --aggregator fedprox --dirichlet 0.5 --dropout
run c5_b 300 python $R --aggregator fedprox
run c5_c 300 python $R --aggregator fedavg --dirichlet 0.5
run c5_e 300 python $R --aggregator fedprox --dirichlet 0.5
run c5_d 500 python $R --aggregator fedprox --dirichlet 0.5 --dropout --no-fused --rounds 8
