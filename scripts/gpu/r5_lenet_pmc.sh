# counters of the LeNet-5 step and fc-grad kernels (config 3)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_lenet_pmc; mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --kernel-include-regex "k_lenet" --output-format csv -d $O/a -o a -- python3 benchmarks/bench_cnn.py --model lenet5 --rounds 1 --warmup 0 --n-train 4096 --n-test 512 > $O/a.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
  --kernel-include-regex "k_lenet" --output-format csv -d $O/b -o b -- python3 benchmarks/bench_cnn.py --model lenet5 --rounds 1 --warmup 0 --n-train 4096 --n-test 512 > $O/b.log 2>&1 || exit 1
