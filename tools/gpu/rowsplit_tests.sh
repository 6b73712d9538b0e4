export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rowsplit.py tests/test_gpu_kernels.py tests/test_gpu_model.py > gpurun_out/rs_tests.log 2>&1
