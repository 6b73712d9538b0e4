# round 5: strided shift sample for the many-component E-step + Morton-ordered columns --
# EM / golden / full-size tests, E-step against sigma, the bench workload's E-step
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05zd
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_atlas_shapes.py tests/test_gpu_multi.py tests/test_gpu_e2e_fullsize.py > gpurun_out/r05zd/tests.log 2>&1
step timeout -k 10 300 python -u tools/probes/estep_sigma.py > gpurun_out/r05zd/estep_sigma.jsonl 2> gpurun_out/r05zd/err
step timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05zd/bench.json 2>> gpurun_out/r05zd/err
echo done
