# round 5: packed-row E/M passes -- bitwise against the scalar rows, the EM tests, the graph
# tests on stable logdet inputs, the A/B (packed 1 / 2 row pairs, scalar, previous build) and
# the host floor.  pytest FAILURES (rc 1) are recorded and the script goes on.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
tstep timeout -k 10 400 $T tests/test_gpu_em.py tests/test_gpu_shoot_graph.py > gpurun_out/r05k_tests.log 2>&1
step timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 2 base lsepk2 lsesc old > gpurun_out/r05k_ab.json 2> gpurun_out/r05k_ab.err
step timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > gpurun_out/r05k_host_floor.txt 2>&1
step timeout -k 10 200 python -u tools/probes/ws_poison.py > gpurun_out/r05k_poison.jsonl 2> gpurun_out/r05k_poison.err
echo done
