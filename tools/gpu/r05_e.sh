# round 5: the 8-row forward rule tests on the final rule, then the W = 4 / 8 gloo rehearsals
# and the PMC passes
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step timeout -k 10 300 $T tests/test_gpu_fwd8.py > gpurun_out/r05e_fwd8.log 2>&1
step bash tools/gpu/r05_rehearse.sh
step bash tools/gpu/r05_pmc.sh
echo done
