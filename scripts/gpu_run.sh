#!/bin/bash
# Parameterised GPU entry point (replaces the one-off gpu_*.sh scripts):
#   OUT=<dir under gpurun_out> bash scripts/gpu_run.sh <step> [<step> ...]
# steps: tests (pytest -m gpu), f32tests (tests/test_mlp_f32_gpu.py), cnntests (tests/test_cnn_engine_gpu.py), smoke, bench (fp32 headline),
#        bench_bf16, bench_cnn, devagg (device SCAFFOLD/FedMedian tests + copy trace),
#        overlap (side-stream / delayed FedAvg tests, bench, kernel overlap trace), prof, stamps,
#        pmc (MLP counters), cnn_configs (BASELINE configs 3-5), cnn_prof (ResNet-18 kernel stats), cnn_pmc (ResNet-18 counters) (rocprofv3 kernel stats of a short fp32 bench), rehearsal (2/4
#        gloo ranks on one GPU). Every GPU step runs under its own time limit; the script stops at
#        the first failure, and at once after a timeout, abort or segfault.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-run}
mkdir -p "$O"
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log"
  fatal $rc "$name"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for step in "$@"; do
  case $step in
    tests) run gpu_tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    f32tests) run f32_tests 400 python -u -m pytest tests/test_mlp_f32_gpu.py -v --timeout 120 --timeout-method thread ;;
    cnntests) run cnn_tests 500 python -u -m pytest tests/test_cnn_engine_gpu.py -v --timeout 150 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench_fp32 300 python bench.py ;;
    bench_bf16) run bench_bf16 300 python bench.py --precision bf16 ;;
    execab)  # A/B: one epoch-graph executable vs two launched alternately
      MYFYP_GRAPH_EXECS=1 run execab_1a 300 python bench.py
      run execab_2a 300 python bench.py
      MYFYP_GRAPH_EXECS=1 run execab_1b 300 python bench.py
      run execab_2b 300 python bench.py ;;
    prepab)  # A/B: epoch gather in the graph vs on the prep stream (overlapping the previous epoch)
      MYFYP_PREP_GATHER=0 run prepab_0a 300 python bench.py
      MYFYP_PREP_GATHER=1 run prepab_1a 300 python bench.py
      MYFYP_PREP_GATHER=0 run prepab_0b 300 python bench.py
      MYFYP_PREP_GATHER=1 run prepab_1b 300 python bench.py ;;
    convab)  # conv operand gathers: raw buffer loads (default) vs pointer loads + selects (build/base_CONV_BUFLOAD0)
      run conv_ab_buf 200 python scripts/probes/conv_ab.py
      MYFYP_NATIVE_LIB=build/base_CONV_BUFLOAD0/libmyfyp_hip.so run conv_ab_base 200 python scripts/probes/conv_ab.py
      run resnet_buf 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      MYFYP_NATIVE_LIB=build/base_CONV_BUFLOAD0/libmyfyp_hip.so run resnet_base 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      run resnet_buf2 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3 ;;
    dmaab)  # forward-shaped convs: LDS-DMA stage ring (default) vs register stage (MYFYP_CONV_DMA=0)
      run conv_ab_dma 300 python scripts/probes/conv_ab.py
      run resnet_dma 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      MYFYP_CONV_DMA=0 run resnet_reg 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      run resnet_dma2 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3 ;;
    dmaprof)  # same-box kernel stats of the ResNet-18 step: register stage (0), DMA forward only (20), DMA forward + wgrad (1)
      for v in 0 20 1; do
        MYFYP_CONV_DMA=$v run cnn_prof_v$v 400 rocprofv3 --kernel-trace --stats -d "$O/cnn_prof_v$v" -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 1 \
          --n-train 16384 --n-test 2048
      done
      for v in 0 20 1; do MYFYP_CONV_DMA=$v run resnet_v$v 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3; done ;;
    statrows)  # BN-statistics atomics spread over 16 accumulator rows vs one (same box, alternating)
      for i in 1 2; do
        MYFYP_BN_STAT_ROWS=1 run resnet_rows1_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        MYFYP_BN_STAT_ROWS=16 run resnet_rows16_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done
      MYFYP_BN_STAT_ROWS=16 run cnn_prof_rows16 400 rocprofv3 --kernel-trace --stats -d "$O/cnn_prof_rows16" -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 1 \
          --n-train 16384 --n-test 2048 ;;
    rowsab)  # spread accumulators (BN forward stats / BN-backward partials): 1 / 16 / 64 rows, alternating
      for i in 1 2; do
        for r in 1 16 64; do MYFYP_BN_STAT_ROWS=$r MYFYP_BNB_ROWS=$r run resnet_r${r}_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3; done
      done ;;
    epiprobe) run conv_epi 300 python scripts/probes/conv_epi_probe.py ;;
    resnet2)
      run resnet_a 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      run resnet_b 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3 ;;
    lenet30)  # config 3 at 30 rounds (the r3b measurement length), twice
      run lenet_ring30_a 400 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30
      run lenet_ring30_b 400 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30 ;;
    lenetab)  # config 3: DMA forward convs (eval path) vs register stage, alternating
      for i in 1 2; do
        MYFYP_CONV_DMA=0 run lenet_reg_$i 400 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30
        MYFYP_CONV_DMA=1 run lenet_dma_$i 400 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 30
      done ;;
    lenetold)  # config 3: the r3b tree (build/r3b_tree, commit 52fcf80) vs this tree, same data flags, alternating
      D="--model lenet5 --aggregator neighbor --rounds 30 --similarity 0.8 --noise 1.2 --modes 4 --label-noise 0.1 --target-acc 0.8"
      for i in 1 2; do
        (cd build/r3b_tree && timeout -k 10 400 python benchmarks/bench_cnn.py $D) > "$O/lenet_old_$i.log" 2>&1 || exit 1
        run lenet_new_$i 400 python benchmarks/bench_cnn.py $D
      done ;;
    wsplit) run wgrad_split 400 python scripts/probes/wgrad_split_sweep.py ;;
    tuneab)  # device-tuned wgrad split-K vs the rule (MYFYP_WGRAD_TUNE=0), alternating
      for i in 1 2; do
        MYFYP_WGRAD_TUNE=0 run resnet_rule_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        run resnet_tuned_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done ;;
    xtab)  # cross-tile DMA prefetch in the forward conv (default) vs one tile at a time (build/base_CONV_XT0), alternating
      L0=build/base_CONV_XT0/libmyfyp_hip.so
      run epi_xt1 300 python scripts/probes/conv_epi_probe.py
      MYFYP_NATIVE_LIB=$L0 run epi_xt0 300 python scripts/probes/conv_epi_probe.py
      for i in 1 2; do
        run resnet_xt1_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        MYFYP_NATIVE_LIB=$L0 run resnet_xt0_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done ;;
    haloab)  # halo wgrad on 64-channel layers only (MAXC=64) vs all 64-multiples (default), alternating
      for i in 1 2; do
        MYFYP_WGRAD_HALO_MAXC=64 run resnet_halo64_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        run resnet_haloall_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done ;;
    halo4ab)  # halo wgrad incl. the 4x4-image layer 4 (default) vs without it (MYFYP_WGRAD_HALO_MAXC=256), alternating
      for i in 1 2; do
        MYFYP_WGRAD_HALO_MAXC=256 run resnet_h256_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        run resnet_hall_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done ;;
    fhaloab)  # layer-1 forward / stride-1 dgrad from one staged patch (default) vs the LDS-DMA kernel (MYFYP_FWD_HALO=0)
      run epi_fh1 300 python scripts/probes/conv_epi_probe.py
      MYFYP_FWD_HALO=0 run epi_fh0 300 python scripts/probes/conv_epi_probe.py
      for i in 1 2; do
        MYFYP_FWD_HALO=0 run resnet_fh0_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        run resnet_fh1_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done ;;
    captab)  # CNN epoch graphs captured in the round that first runs them (default) vs one round later (MYFYP_CNN_CAPTURE_LATE=1)
      for i in 1 2; do
        MYFYP_CNN_CAPTURE_LATE=1 run resnet_late_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
        run resnet_early_$i 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      done
      MYFYP_CNN_CAPTURE_LATE=1 run lenet_late 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 20
      run lenet_early 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 20 ;;
    onepeer)  # the device work of one rank of the N=8 / N=4 runs: 1 / 2 peers of 7.5k samples each on one GPU (no RCCL)
      run onepeer_p1 300 python bench.py --peers 1 --n-train 7500 --n-test 1250
      run onepeer_p2 300 python bench.py --peers 2 --n-train 15000 --n-test 2500 ;;
    bench_cnn) run bench_cnn 600 python benchmarks/bench_cnn.py ;;
    apitrace)  # HIP API + kernel + copy trace of a short fp32 bench: GPU idle gaps and host-blocking calls
      run apitrace 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "$O/api" -o run -- python3 bench.py --steps 40 --warmup 5
      python3 scripts/tools/api_blocking.py "$O"/api > "$O/api_blocking.txt" 2>&1; cat "$O/api_blocking.txt" ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python bench.py --steps 40 --warmup 5 ;;
    devagg)
      run devagg_tests 300 python -u -m pytest tests/test_device_aggregators.py tests/test_kernels_gpu.py -k "device_plane or median" -v -m gpu --timeout 120 --timeout-method thread
      run devagg_prof 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/agg" -o run -- python3 scripts/probes/device_agg_copies.py
      mv gpurun_out/device_agg_windows.json "$O/" && python3 scripts/tools/copies_in_window.py "$O"/agg/run_results.db "$O/device_agg_windows.json" > "$O/devagg_windows.txt"
      cat "$O/devagg_windows.txt" ;;
    overlap)
      run overlap_tests 400 python -u -m pytest tests/test_overlap.py tests/test_cnn_engine_gpu.py -k "overlap or delayed or lenet_fused_epoch" -v -m gpu --timeout 120 --timeout-method thread
      run bench_cnn_delayed 600 python benchmarks/bench_cnn.py --delayed-averaging
      run overlap_prof 300 rocprofv3 --kernel-trace -d "$O/ovl" -o run -- python3 scripts/probes/overlap_probe.py
      python3 scripts/tools/kernel_overlap.py "$O"/ovl/run_results.db fedavg > "$O/overlap.txt"; cat "$O/overlap.txt" ;;
    stamps)  # phase timestamps of the fp32 persistent epoch (library built with: python -m myfyp_amd.ops.build --stamps)
      MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so run stamps_f32 200 python scripts/probes/stamps_f32.py ;;
    pmc)  # counters of the MLP kernels, one pass per counter group (never with a trace domain)
      run pmc_a 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
        --kernel-include-regex "mlp_" --output-format csv -d "$O/pmc_a" -o a -- python3 bench.py --steps 2 --warmup 1
      run pmc_b 300 timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum \
        --kernel-include-regex "mlp_" --output-format csv -d "$O/pmc_b" -o b -- python3 bench.py --steps 2 --warmup 1 ;;
    cnn_configs)  # BASELINE configs 3, 4, 5
      run lenet_ring 400 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 20
      run resnet_fedavg 400 python benchmarks/bench_cnn.py --model resnet18 --rounds 3
      run resnet_fedprox_drop 400 python benchmarks/bench_cnn.py --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 3 ;;
    cnn_pmc)  # counters of the ResNet-18 conv / BN / optimizer kernels, one pass per counter group
      run cnn_pmc_a 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
        --kernel-include-regex "k_conv|k_bn|k_opt" --output-format csv -d "$O/cnn_pmc_a" -o a -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 0 --n-train 2048 --n-test 512
      run cnn_pmc_b 300 timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
        --kernel-include-regex "k_conv|k_bn|k_opt" --output-format csv -d "$O/cnn_pmc_b" -o b -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 0 --n-train 2048 --n-test 512 ;;
    cnn_prof)  # kernel statistics of the ResNet-18 grouped step
      run cnn_prof 400 rocprofv3 --kernel-trace --stats -d "$O/cnn_prof" -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --warmup 1 \
        --n-train 16384 --n-test 2048 ;;
    cnn_round_prof)  # kernel trace of full-size config-4 rounds (round boundary: evaluation, FedAvg, host gaps)
      run cnn_round_prof 400 rocprofv3 --kernel-trace -d "$O/cnn_round_prof" -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 2 --warmup 1 ;;
    rehearsal)
      for n in ${REHEARSAL_NS:-2 4}; do
        MYFYP_DIST_BACKEND=gloo run rehearsal_gloo_n$n 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port 2970$n bench.py --gpus $n --steps 10 --warmup 2
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
