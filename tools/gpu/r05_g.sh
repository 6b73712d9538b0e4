# round 5: host floor at 2k points (tools/host_floor.py) and its cProfile breakdown
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 300 python -u tools/host_floor.py --sizes 2000 --iters 3 > gpurun_out/r05g_host_floor.txt 2>&1
step timeout -k 10 300 python -u tools/host_profile.py --N 2000 > gpurun_out/r05g_host_profile.txt 2>&1
echo done
