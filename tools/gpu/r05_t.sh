# round 5: per-pair re-referencing in the LSE passes -- E-step time against sigma (with / without
# the shift hint), EM tests, A/B line
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_sigma.py > gpurun_out/r05t_estep_sigma.jsonl 2> gpurun_out/r05t.err
tstep timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_atlas_shapes.py tests/test_gpu_multi.py tests/test_gpu_fullsize.py > gpurun_out/r05t_tests.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 2 base > gpurun_out/r05t_ab.json 2>> gpurun_out/r05t.err
echo done
