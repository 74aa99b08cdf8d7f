set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=3 timeout -k 10 200 python scripts/probes/stamps_f32v3.py > gpurun_out/st3.log 2>&1
for mode in 2 0; do
  MYFYP_PREP_GATHER=$mode timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g$mode -o run -- python bench.py --steps 60 --warmup 5 > gpurun_out/bench_g$mode.log 2>&1
done
