# round 5: pair-once centred KRed (sym_cx.hpp) and the 8-row symmetric forward: parity + timing
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 400 $T tests/test_gpu_sym_red.py "tests/test_gpu_centred.py::test_kernel_sum_100k_fullsize" > gpurun_out/r05_sym.log 2>&1
step timeout -k 10 400 $T tests/test_gpu_fwd8.py > gpurun_out/r05_fwd8.log 2>&1
step timeout -k 10 300 python -u tools/probes/sym_red_ab.py 0 1 2 4 > gpurun_out/r05_sym_ab.jsonl 2> gpurun_out/r05_sym_ab.err
step timeout -k 10 300 python -u tools/probes/fwd8_ab.py > gpurun_out/r05_fwd8_ab.jsonl 2> gpurun_out/r05_fwd8_ab.err
step timeout -k 10 400 $T tests/test_gpu_multi.py > gpurun_out/r05_multi.log 2>&1
step timeout -k 10 700 $T tests/test_gpu_e2e_fullsize.py -k logdet > gpurun_out/r05_e2e_logdet.log 2>&1
