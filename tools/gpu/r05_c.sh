# round 5: 4 / 8-row pair-once KRed and the 8-row forward: parity + geometry sweeps;
# multi-structure traces and the logdet e2e with the adjusted criteria
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 400 $T tests/test_gpu_sym_red.py > gpurun_out/r05c_sym.log 2>&1
step timeout -k 10 300 python -u tools/probes/sym_red_ab.py 4:0 4:2 8:0 8:1 8:2 > gpurun_out/r05c_sym_ab.jsonl 2> gpurun_out/r05c_sym_ab.err
step timeout -k 10 300 python -u tools/probes/fwd8_ab.py > gpurun_out/r05c_fwd8_ab.jsonl 2> gpurun_out/r05c_fwd8_ab.err
step timeout -k 10 400 $T tests/test_gpu_multi.py > gpurun_out/r05c_multi.log 2>&1
step timeout -k 10 700 $T tests/test_gpu_e2e_fullsize.py -k logdet > gpurun_out/r05c_e2e_logdet.log 2>&1
