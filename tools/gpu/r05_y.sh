# round 5: the adaptive re-reference threshold (lse_adapt) with the clamped-share start -- E-step against sigma, and the
# bench workload's own E-step time per threshold
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05y
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 300 python -u tools/probes/estep_sigma.py > gpurun_out/r05y_estep_sigma.jsonl 2> gpurun_out/r05y.err
for a in 1 1000; do
  DICP_LSE_ADAPT=$a step timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05y/bench_a$a.json 2>> gpurun_out/r05y.err
done
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_em.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_atlas_shapes.py > gpurun_out/r05y_tests.log 2>&1; echo tests rc=$?
echo done
