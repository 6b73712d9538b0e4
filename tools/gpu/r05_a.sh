# round 5: multi-structure traces + C5 iteration, EM single sweep, final-shoot completion,
# eta != 0 / 0.5 sigma full-size e2e, a bench line
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
# a test FAILURE (rc 1) goes on to the next step; a fault / abort / time limit stops the script
step() { "$@"; rc=$?; case $rc in 0|1) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 400 $T tests/test_gpu_multi.py > gpurun_out/r05_multi.log 2>&1
step timeout -k 10 400 $T tests/test_gpu_em.py tests/test_gpu_atlas_shapes.py "tests/test_gpu_golden.py::test_em_golden" -k "not c4_iteration" > gpurun_out/r05_em.log 2>&1
step timeout -k 10 400 $T tests/test_gpu_model.py -k "final_shoot" > gpurun_out/r05_final_shoot.log 2>&1
step timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r05_bench.log 2>&1
step timeout -k 10 700 $T tests/test_gpu_e2e_fullsize.py > gpurun_out/r05_e2e.log 2>&1
