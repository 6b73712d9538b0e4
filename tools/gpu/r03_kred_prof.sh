# Kernel trace + SQ issue / LDS counters of the centred KRed (100k x 100k, x = y) alone
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PMC_OPS=kred
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kred_kt -o kt --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/kred_kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/kred_issue -o issue --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/kred_issue.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/kred_lds -o lds --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/kred_lds.log 2>&1
python3 tools/pmc_issue.py gpurun_out/kred_issue > gpurun_out/kred_issue.json
