# Node.start breakdown (prewarm) and a driver cProfile of the 8-member virtual mesh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probes/start_breakdown.py > gpurun_out/start_a.log 2>&1
timeout -k 10 200 python scripts/probes/start_breakdown.py > gpurun_out/start_b.log 2>&1
MYFYP_PROFILE_DRIVER=gpurun_out/drv_v8.prof timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --steps 100 --warmup 10 > gpurun_out/bench_virt8_prof.log 2>&1
python scripts/probes/driver_profile_summary.py gpurun_out/drv_v8.prof > gpurun_out/drv_v8.txt 2>&1
MYFYP_PROFILE_DRIVER=gpurun_out/drv_n1.prof timeout -k 10 200 python bench.py --steps 200 --warmup 10 > gpurun_out/bench_n1_prof.log 2>&1
python scripts/probes/driver_profile_summary.py gpurun_out/drv_n1.prof > gpurun_out/drv_n1.txt 2>&1
