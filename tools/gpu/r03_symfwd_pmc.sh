# SQ issue counters of the ordered (fwd_alg 2) vs symmetric (fwd_alg 4) packed forward at 100k
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PMC_OPS=symfwd
O=gpurun_out/r03sf
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/issue -o issue --output-format csv -- python3 tools/pmc_probe.py > $O/issue.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM -d $O/lds -o lds --output-format csv -- python3 tools/pmc_probe.py > $O/lds.log 2>&1
python3 tools/pmc_issue.py $O/issue > $O/issue.json
echo done
