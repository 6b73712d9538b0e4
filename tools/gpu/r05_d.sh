# round 5: ring-LDS pair-once KRed (parity + A/B against the no-ring build), the 8-row forward
# at 3 waves / SIMD (A/B), the automatic geometry of the pair-once KRed
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 400 $T tests/test_gpu_sym_red.py tests/test_gpu_centred.py > gpurun_out/r05d_sym.log 2>&1
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 3 base scxnoring > gpurun_out/r05d_ab_ring.json 2> gpurun_out/r05d_ab_ring.err
DICP_AB_OPTS=sym_fwd_rows=8,sym_L=1 step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 3 base fwd8w3 > gpurun_out/r05d_ab_fwd8w3.json 2> gpurun_out/r05d_ab_fwd8w3.err
DICP_AB_OPTS=sym_fwd_rows=4 step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 3 base > gpurun_out/r05d_ab_fwd4.json 2> gpurun_out/r05d_ab_fwd4.err
step timeout -k 10 300 python -u tools/probes/sym_red_ab.py 4:0 > gpurun_out/r05d_sym_ab.jsonl 2> gpurun_out/r05d_sym_ab.err
