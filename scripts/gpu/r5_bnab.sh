# fuse_fin test after the ticket ordering fix; ResNet-18 config 4 with / without the generic BN1 prologue fold
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_bnab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "finalize_in_conv_tail or one_step or lenet" > $O/cnn_fin.log 2>&1
for i in a b; do
  timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1 > $O/rn_base_$i.log 2>&1
  MYFYP_CNN_FUSE_BN=1 timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1 > $O/rn_fusebn_$i.log 2>&1
done
