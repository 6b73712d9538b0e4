# symmetric VJP column groups per workgroup L = 8 (default at 100k) vs 12 / 16 / 24: time
# (alternating, one process) and PMC write / fetch traffic per launch (separate passes)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03l2
mkdir -p $O
SYM_LS=8,12,16,24 timeout -k 10 200 python tools/symL_ab.py > $O/symL_ab.json 2> $O/symL_ab.err
for L in 8 16; do
  PMC_SYM_L=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc$L -o fetch --output-format csv -- python3 tools/pmc_probe.py > $O/fetch$L.log 2>&1
  PMC_SYM_L=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc$L -o write --output-format csv -- python3 tools/pmc_probe.py > $O/write$L.log 2>&1
done
echo done
