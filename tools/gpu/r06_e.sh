set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_em.py tests/test_gpu_rowsplit.py tests/test_gpu_golden.py -q --timeout 300 --timeout-method thread > gpurun_out/r06_e.log 2>&1
timeout -k 10 120 python -u tools/probes/rowsplit_fe.py > gpurun_out/r06_rowsplit_fe2.jsonl 2>> gpurun_out/r06_e.err
DICP_ESTEP_HINT_ANY=1 timeout -k 10 120 python -u tools/probes/rowsplit_fe.py >> gpurun_out/r06_rowsplit_fe2.jsonl 2>> gpurun_out/r06_e.err
