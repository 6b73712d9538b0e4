set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probes/logdet_cost_diag.py --M 20000 --steps 0 > gpurun_out/r06_logdet_diag20k_fix.jsonl 2> gpurun_out/r06_fix.err
timeout -k 10 300 python -u tools/probes/logdet_cost_diag.py vsrc --M 20000 > gpurun_out/r06_logdet_vsrc20k_fix.jsonl 2>> gpurun_out/r06_fix.err
for s in grid decim; do for w in 0 1; do timeout -k 10 200 python -u tools/probes/psr_std_trace.py $s $w >> gpurun_out/r06_psr_std_trace.jsonl 2>> gpurun_out/r06_fix.err || exit 1; done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_fullsize.py -k logdet -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r06_e2e_logdet_fix.log 2>&1
