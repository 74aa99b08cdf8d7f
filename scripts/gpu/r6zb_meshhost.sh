# Host cost per round of the device-mesh round driver without GPU back-pressure: 8 virtual mesh
# members on one GPU with tiny epochs (the GPU then waits for the host, so the driver's CPU time is
# its own work, not spinning on a full launch queue), against the same work in one group.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6zb_meshhost; mkdir -p $O
for nt in 4096 60000; do
  timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --n-train $nt --n-test 1024 --steps 100 --warmup 5 > $O/mesh8_$nt.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --n-train $nt --n-test 1024 --steps 100 --warmup 5 > $O/one_$nt.log 2>&1 || exit 1
done
MYFYP_PROFILE_DRIVER=$O/mesh8_small.prof timeout -k 10 200 python bench.py --gpus 8 --mesh-virtual --n-train 4096 --n-test 1024 --steps 100 --warmup 5 > $O/mesh8_small_prof.log 2>&1 || exit 1
grep -h "driver_round_cpu" $O/*.log
for f in $O/mesh8_*.log $O/one_*.log; do echo $f $(tail -n 1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"); done
