# round 5: the adaptive re-reference threshold (lse_adapt) -- E-step against sigma, and the
# bench workload's own E-step time per threshold
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05w
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 300 python -u tools/probes/estep_sigma.py > gpurun_out/r05w_estep_sigma.jsonl 2> gpurun_out/r05w.err
for a in 0 1 4 1000; do
  DICP_LSE_ADAPT=$a step timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05w/bench_a$a.json 2>> gpurun_out/r05w.err
done
echo done
