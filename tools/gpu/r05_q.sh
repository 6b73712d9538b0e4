# round 5: the uniform-weight E-step at the Chui two-set shapes; the Chui trace with this build
# and with the committed one
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_uniform.py > gpurun_out/r05q_uniform.jsonl 2> gpurun_out/r05q_uniform.err
DICP_LIB_PATH=diff-icp_amd/variants/libdifficp_hip_nouni.so step timeout -k 10 200 python -u tools/probes/estep_uniform.py > gpurun_out/r05q_uniform_nouni.jsonl 2>> gpurun_out/r05q_uniform.err
tstep timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_golden.py -k chui > gpurun_out/r05q_chui.log 2>&1
DICP_LIB_PATH=diff-icp_amd/variants/libdifficp_hip_nouni.so tstep timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_golden.py -k chui > gpurun_out/r05q_chui_nouni.log 2>&1
echo done
