# ResNet-18 (config 4): weight gradients on a side-stream graph branch vs one stream (alternating),
# then the CNN engine GPU tests on the new default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f_wgstream; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/one_$i.log 2>&1 || exit 1
  MYFYP_CNN_WGRAD_STREAM=1 timeout -k 10 300 python benchmarks/bench_cnn.py --model resnet18 --rounds 10 > $O/side_$i.log 2>&1 || exit 1
done
for f in $O/one_*.log $O/side_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_round"], d["final_test_acc_mean"])')"; done
MYFYP_CNN_WGRAD_STREAM=1 timeout -k 10 900 python -u -m pytest tests/test_cnn_engine_gpu.py -x -q --timeout 300 --timeout-method thread > $O/cnn_tests.log 2>&1 || exit 1
tail -3 $O/cnn_tests.log
