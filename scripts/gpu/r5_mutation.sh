# Mutation check: every fused-engine update scaled by 1.05 (MYFYP_DEBUG_LR_SCALE);
# which tests notice? Each step is allowed to fail; the summary lines are what matter.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_mutation; mkdir -p $O
export MYFYP_DEBUG_LR_SCALE=1.05
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" > $O/summary.txt
timeout -k 10 600 python -u -m pytest tests/test_cnn_engine_gpu.py -q --timeout 300 --timeout-method thread -k "one_step or matches_materialised or conv_tail or parity_forward or fused_epoch" > $O/cnn.log 2>&1; echo "cnn rc=$?" >> $O/summary.txt
timeout -k 10 600 python -u -m pytest tests/test_mlp_f32_gpu.py -q --timeout 300 --timeout-method thread -k "not prep_stream" > $O/mlp.log 2>&1; echo "mlp rc=$?" >> $O/summary.txt
timeout -k 10 700 python -u -m pytest tests/test_config5_gpu.py -q --timeout 600 --timeout-method thread > $O/config5.log 2>&1; echo "config5 rc=$?" >> $O/summary.txt
exit 0
