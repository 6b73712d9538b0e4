# round-2 validation + profiles: full GPU suite, headline bench, rocprofv3 kernel stats of the
# same command, PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ/GRBM issue pass
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_issue.log 2>&1
echo done
