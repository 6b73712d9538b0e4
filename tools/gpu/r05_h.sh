# round 5: branch-free single-sweep E/M passes (EM parity, A/B vs the committed build and the
# 4-row variant), HIP-graph shooting replay (bitwise tests, host floor + profile at 2k), the
# 8-row forward rule; then the W = 4 / 8 rehearsals and the PMC passes
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step timeout -k 10 300 $T tests/test_gpu_shoot_graph.py > gpurun_out/r05h_graph.log 2>&1
step timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > gpurun_out/r05h_host_floor.txt 2>&1
step timeout -k 10 200 python -u tools/host_profile.py --N 2000 > gpurun_out/r05h_host_profile.txt 2>&1
step timeout -k 10 500 $T tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_atlas_shapes.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multi.py tests/test_gpu_fwd8.py > gpurun_out/r05h_tests.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 2 base old lse4 > gpurun_out/r05h_ab_em.json 2> gpurun_out/r05h_ab_em.err
step bash tools/gpu/r05_rehearse.sh
step bash tools/gpu/r05_pmc.sh
echo done
