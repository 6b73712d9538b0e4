# round 5: the 2D eta != 0 VJP NaN (variants and the float64 oracle), the packed / scalar E-M
# bitwise test after the pair-recovery fix, the E-step row pairs per pass
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
step timeout -k 10 300 python -u tools/probes/logdet2d_nan.py > gpurun_out/r05l_logdet2d.jsonl 2> gpurun_out/r05l_logdet2d.err
tstep timeout -k 10 300 $T tests/test_gpu_em.py > gpurun_out/r05l_em.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 2 base > gpurun_out/r05l_ab.json 2> gpurun_out/r05l_ab.err
echo done
