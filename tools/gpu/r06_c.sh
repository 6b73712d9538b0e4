set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probes/logdet_cost_diag.py vsrc --M 20000 > gpurun_out/r06_logdet_vsrc20k_f64.jsonl 2> gpurun_out/r06_c.err
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_fullsize.py -k logdet -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r06_e2e_logdet_f64.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize_eta.py tests/test_gpu_golden.py tests/test_gpu_api.py tests/test_gpu_rowsplit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c_tests.log 2>&1
