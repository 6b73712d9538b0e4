# round 5: the branch-free single-sweep E/M passes -- EM parity (direct E-step stats, goldens,
# atlas shapes, full-size rows, multi-structure traces), the A/B against the committed build
# and the 4-row variant, the 8-row forward rule tests; then the W = 4 / 8 rehearsals and PMC
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step timeout -k 10 600 $T tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_atlas_shapes.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multi.py tests/test_gpu_support.py tests/test_gpu_fwd8.py > gpurun_out/r05f_tests.log 2>&1
step timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 3 base old lse4 > gpurun_out/r05f_ab_em.json 2> gpurun_out/r05f_ab_em.err
step bash tools/gpu/r05_rehearse.sh
step bash tools/gpu/r05_pmc.sh
echo done
