# SQ/GRBM issue counters of the hot kernels at the bench's sizes (two separate --pmc passes)
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_issue.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc_lds -o lds --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/pmc_lds.log 2>&1
