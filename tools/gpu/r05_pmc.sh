# round 5: SQ/GRBM issue counters of the hot kernels (the 8-row forward, the 4-row VJP, the
# E-step) and of the kernel sum (pair-once x = y, ordered x != y); traffic passes separately
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ISSUE="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $ISSUE -d gpurun_out/r05_pmc_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmc_issue.log 2>&1
PMC_OPS=ksum timeout -s KILL 120 rocprofv3 --pmc $ISSUE -d gpurun_out/r05_pmc_ksum -o ksum --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmc_ksum.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r05_pmc_traffic -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r05_pmc_traffic -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/r05_pmc_write.log 2>&1
python3 tools/pmc_issue.py gpurun_out/r05_pmc_issue > gpurun_out/r05_pmc_issue.json
python3 tools/pmc_issue.py gpurun_out/r05_pmc_ksum > gpurun_out/r05_pmc_ksum.json
python3 tools/pmc_traffic.py gpurun_out/r05_pmc_traffic > gpurun_out/r05_pmc_traffic.json
