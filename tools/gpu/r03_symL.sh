# round 3: symmetric VJP column groups per workgroup L = 4 vs 8 (the new default at 100k):
# time (alternating, one process) and PMC write / fetch traffic per launch (separate passes)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r03l
timeout -k 10 200 python tools/symL_ab.py > gpurun_out/r03l/symL_ab.json 2> gpurun_out/r03l/symL_ab.err
for L in 4 8; do
  PMC_SYM_L=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03l/pmc$L -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r03l/fetch$L.log 2>&1
  PMC_SYM_L=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r03l/pmc$L -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r03l/write$L.log 2>&1
done
echo done
