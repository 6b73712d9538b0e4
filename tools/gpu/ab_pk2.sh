export PYTHONUNBUFFERED=1
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "ode_self_fwd or ode_self_bwd or sym_bwd or euler" > gpurun_out/pk2_tests.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 2 base pkpf pkpfu1 > gpurun_out/ab_pk2_100k.json 2> gpurun_out/ab_pk2.err
timeout -k 10 200 python -u tools/ab_tune.py --mode fwdeta --M 50000 --rounds 5 > gpurun_out/ab_fwdeta.json 2>> gpurun_out/ab_pk2.err
