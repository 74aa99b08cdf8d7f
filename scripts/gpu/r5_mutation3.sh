# the CNN one-step tests with the aggregate update-scale check: clean, then with the 5 % mutation
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_mutation3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cnn_engine_gpu.py -q --timeout 300 --timeout-method thread -k "train_step_matches_torch" -rA > $O/cnn_clean.log 2>&1; echo "cnn clean rc=$?" > $O/summary.txt
MYFYP_DEBUG_LR_SCALE=1.05 timeout -k 10 600 python -u -m pytest tests/test_cnn_engine_gpu.py -q --timeout 300 --timeout-method thread -k "train_step_matches_torch" > $O/cnn_mut.log 2>&1; echo "cnn mutated rc=$?" >> $O/summary.txt
cat $O/summary.txt
exit 0
