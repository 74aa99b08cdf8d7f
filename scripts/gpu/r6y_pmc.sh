# Counters of the headline's fp32 persistent epoch on the late round-6 tree (one-round-trip polls,
# shortened softmax), same passes as scripts/gpu/r5_mlp_pmc.sh (default hand-offs only).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6y_pmc; mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/a -o a -- python3 bench.py --steps 3 --warmup 2 > $O/a.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
  --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/b -o b -- python3 bench.py --steps 3 --warmup 2 > $O/b.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum \
  --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/c -o c -- python3 bench.py --steps 3 --warmup 2 > $O/c.log 2>&1 || exit 1
python3 scripts/probes/pmc_summary.py $(find $O/a $O/b $O/c -name '*counter_collection.csv') > $O/pmc.txt
cat $O/pmc.txt
