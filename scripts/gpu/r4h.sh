#!/bin/bash
# round 4, call H: gather-ahead mode (MYFYP_PREP_GATHER=2) A/B; Adam+extra layout routing (v1 spilled vs v2)
set -o pipefail
O=gpurun_out/r4h; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -4 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
run test_prep 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_f32_gpu.py -k "prep or prox or scaffold or extra"
AGG=fedprox run prox_auto 200 python scripts/probes/epoch_f32_extra.py
AGG=fedprox MYFYP_F32_VARIANT=1 run prox_v1 200 python scripts/probes/epoch_f32_extra.py
AGG=scaffold run scaf_auto 200 python scripts/probes/epoch_f32_extra.py
AGG=scaffold MYFYP_F32_VARIANT=1 run scaf_v1 200 python scripts/probes/epoch_f32_extra.py
AGG=fedavg run avg_auto 200 python scripts/probes/epoch_f32_extra.py
run bench_base_a 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=2 run bench_prep2_a 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=2 MYFYP_PREP_GATHER_WGS=32 run bench_prep2w32_a 200 python bench.py --steps 200 --warmup 10
run bench_base_b 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=2 run bench_prep2_b 200 python bench.py --steps 200 --warmup 10
MYFYP_PREP_GATHER=1 run bench_prep1 200 python bench.py --steps 200 --warmup 10
