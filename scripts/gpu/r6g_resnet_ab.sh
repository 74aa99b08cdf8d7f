# ResNet-18 (config 4) A/B in one call: halo wgrad prefetch depth 1 vs 2 (default 2), and the
# weight gradients on a side-stream graph branch (opt-in) — arms alternating — then the CNN engine
# GPU tests with the side stream on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g_resnet_ab; mkdir -p $O
run() { timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/$1.log 2>&1; }
for i in 1 2; do
  MYFYP_WGRAD_PF=1 run pf1_$i || exit 1
  run pf2_$i || exit 1
  MYFYP_CNN_WGRAD_STREAM=1 run side_$i || exit 1
done
for f in $O/pf*.log $O/side_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_round"], d["final_test_acc_mean"])')"; done
MYFYP_CNN_WGRAD_STREAM=1 timeout -k 10 900 python -u -m pytest tests/test_cnn_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1 || exit 1
tail -3 $O/cnn_tests.log
