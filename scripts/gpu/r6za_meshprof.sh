# Host cost of the device-mesh round driver: cProfile of the driver thread with 8 virtual mesh
# members on one GPU (MYFYP_PROFILE_DRIVER), plus the one-group headline for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6za_meshprof; mkdir -p $O
MYFYP_PROFILE_DRIVER=$O/mesh8.prof timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --steps 50 --warmup 5 > $O/mesh8.log 2>&1 || exit 1
MYFYP_PROFILE_DRIVER=$O/one.prof timeout -k 10 200 python bench.py --steps 50 --warmup 5 > $O/one.log 2>&1 || exit 1
python - <<'PY' > $O/pstats.txt
import pstats
for f in ("gpurun_out/r6za_meshprof/mesh8.prof", "gpurun_out/r6za_meshprof/one.prof"):
    print("=====", f)
    s = pstats.Stats(f); s.sort_stats("tottime").print_stats(40)
    s.sort_stats("cumulative").print_stats(50)
PY
tail -n 1 $O/mesh8.log | cut -c1-200
