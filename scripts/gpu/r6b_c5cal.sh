# Round 6 (second session): headline sanity on the rebuilt tree, then the config-5 calibration
# runs for the test's fixed bounds (three engine seeds, three torch seeds, two mutated engine seeds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6b_c5cal; mkdir -p $O
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench20.log 2>&1 || exit 1
timeout -k 10 800 python -u scripts/probes/config5_calibrate2.py e1 e2 e3 t1 t2 t3 > $O/c5_clean.log 2>&1 || exit 1
MYFYP_DEBUG_LR_SCALE=1.05 timeout -k 10 400 python -u scripts/probes/config5_calibrate2.py e1 e2 e3 > $O/c5_mut.log 2>&1 || exit 1
tail -1 $O/bench20.log; grep scale= $O/c5_clean.log $O/c5_mut.log
