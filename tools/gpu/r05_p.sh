# round 5: uniform-weight tiles in the E-step -- EM tests, A/B against the committed build
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 200 --timeout-method thread"
tstep timeout -k 10 400 $T tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py > gpurun_out/r05p_tests.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 3 base nouni > gpurun_out/r05p_ab.json 2> gpurun_out/r05p_ab.err
echo done
