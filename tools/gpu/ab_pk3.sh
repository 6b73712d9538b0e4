export PYTHONUNBUFFERED=1
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rowsplit.py -k "bwd or fwd or euler or sym" > gpurun_out/pk3_tests.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 3 base prev > gpurun_out/ab_pk3_100k.json 2> gpurun_out/ab_pk3.err
timeout -k 10 200 python -u tools/ab_tune.py --mode eta --M 50000 --rounds 5 > gpurun_out/ab_eta.json 2>> gpurun_out/ab_pk3.err
