set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
DICP_LIB_PATH=$PWD/diff-icp_amd/variants/libdifficp_hip_ldsacc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bwd" > gpurun_out/ldsacc_tests.log 2>&1 || { tail -30 gpurun_out/ldsacc_tests.log; exit 1; }
tail -1 gpurun_out/ldsacc_tests.log
timeout -k 10 400 python -u tools/ab_libs.py --M 100000 --passes 3 base ldsacc > gpurun_out/ab_ldsacc100k.json 2> gpurun_out/ab_ldsacc.err
cat gpurun_out/ab_ldsacc100k.json
timeout -k 10 400 python -u tools/ab_libs.py --M 50000 --passes 3 base ldsacc > gpurun_out/ab_ldsacc50k.json 2>> gpurun_out/ab_ldsacc.err
cat gpurun_out/ab_ldsacc50k.json
