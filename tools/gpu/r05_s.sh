# round 5: E-step time against sigma with / without the shift hint; EM tests; the kernel-sum probes
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_sigma.py > gpurun_out/r05s_estep_sigma.jsonl 2> gpurun_out/r05s.err
tstep timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_atlas_shapes.py tests/test_gpu_multi.py tests/test_lib_load.py > gpurun_out/r05s_tests.log 2>&1
step timeout -k 10 200 python -u tools/probes/sym_red_ab.py 4:0 > gpurun_out/r05s_sym_ab.jsonl 2>> gpurun_out/r05s.err
echo done
