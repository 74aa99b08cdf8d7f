# Attribution of the 1-GPU N-rank rehearsal (the torchrun one-process-per-GPU path sharing one card)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_ranks; mkdir -p $O
MYFYP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 4 --launch ranks --steps 30 --warmup 5 > $O/ranks4.log 2>&1
MYFYP_DIST_BACKEND=gloo timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace4 -o run -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --launch ranks --steps 30 --warmup 5 > $O/ranks4_trace.log 2>&1
