# counters of the headline's fp32 persistent epoch, single-XCD hand-offs on (default) vs off, plus kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_mlp_pmc; mkdir -p $O
for v in 1 0; do
  MYFYP_F32_PLAIN_PUB=$v timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/a$v -o a -- python3 bench.py --steps 3 --warmup 2 > $O/a$v.log 2>&1 || exit 1
  MYFYP_F32_PLAIN_PUB=$v timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
    --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/b$v -o b -- python3 bench.py --steps 3 --warmup 2 > $O/b$v.log 2>&1 || exit 1
  MYFYP_F32_PLAIN_PUB=$v timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    --kernel-include-regex "mlp_persistent_f32_epoch" --output-format csv -d $O/c$v -o c -- python3 bench.py --steps 3 --warmup 2 > $O/c$v.log 2>&1 || exit 1
  python3 scripts/probes/pmc_summary.py $(find $O/a$v $O/b$v $O/c$v -name '*counter_collection.csv') > $O/pmc_plain$v.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 40 --warmup 5 > $O/stats.log 2>&1 || exit 1
find $O/stats -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
D=$(find $O/stats -name '*.db' | head -1)
[ -n "$D" ] && python3 scripts/probes/rocpd_timeline.py "$D" k_eval_snapshot 30 seq > $O/timeline_direct.txt
find $O -name '*.db' -delete
cat $O/pmc_plain1.txt $O/pmc_plain0.txt
