set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "ode_self_bwd or sym_bwd_vs_ordered" > gpurun_out/pk_tests.log 2>&1
timeout -k 10 200 python -u tools/ab_tune.py --mode pk --M 100000 --rounds 5 > gpurun_out/pk_ab100k.json 2> gpurun_out/pk_ab.err
timeout -k 10 200 python -u tools/ab_tune.py --mode pk --M 50000 --rounds 5 > gpurun_out/pk_ab50k.json 2>> gpurun_out/pk_ab.err
