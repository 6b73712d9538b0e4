export PYTHONUNBUFFERED=1
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rowsplit.py -k "bwd or sym" > gpurun_out/merge_tests.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 3 base prev > gpurun_out/ab_merge.json 2> gpurun_out/ab_merge.err
