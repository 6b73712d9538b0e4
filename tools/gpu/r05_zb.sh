# round 5: normalised store of extreme chunk partials (stale-high shift hints) -- the hint
# offset probe, the EM / golden / full-size tests, the bench workload's E-step
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05zb
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_hint_debug.py > gpurun_out/r05zb/hint_debug.jsonl 2>&1
step timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_atlas_shapes.py tests/test_gpu_multi.py > gpurun_out/r05zb/tests.log 2>&1
step timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05zb/bench.json 2> gpurun_out/r05zb/err
echo done
