# round 5: the lockstep-batch tests after the workspace-cache fix, with the graph / model tests
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 200 --timeout-method thread"
tstep timeout -k 10 600 $T tests/test_gpu_batch.py tests/test_gpu_shoot_graph.py tests/test_gpu_model.py > gpurun_out/r05n_tests.log 2>&1
echo done
