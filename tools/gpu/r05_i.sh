# round 5: workspace-poison probe (kernels reading unwritten workspace?), then the EM / graph /
# host-floor checks, the A/B, the rehearsals and the PMC passes.  A pytest FAILURE (rc 1) is
# recorded and the script goes on; any other status (fault, abort, time limit) stops it.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
step timeout -k 10 200 python -u tools/probes/ws_poison.py > gpurun_out/r05i_poison.jsonl 2> gpurun_out/r05i_poison.err
tstep timeout -k 10 300 $T tests/test_gpu_shoot_graph.py > gpurun_out/r05i_graph.log 2>&1
step timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > gpurun_out/r05i_host_floor.txt 2>&1
step timeout -k 10 200 python -u tools/host_profile.py --N 2000 > gpurun_out/r05i_host_profile.txt 2>&1
tstep timeout -k 10 500 $T -x tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_atlas_shapes.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multi.py tests/test_gpu_fwd8.py > gpurun_out/r05i_tests.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 2 base old lse4 > gpurun_out/r05i_ab_em.json 2> gpurun_out/r05i_ab_em.err
step bash tools/gpu/r05_rehearse.sh
step bash tools/gpu/r05_pmc.sh
echo done
