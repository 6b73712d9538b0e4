# round 5: direct loss-grad closures + graphs -- bitwise tests (graph, Optimize, concurrent
# frames vs sequential), the model / atlas / multi-structure suites, then the host floor
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 200 --timeout-method thread"
tstep timeout -k 10 700 $T tests/test_gpu_shoot_graph.py tests/test_gpu_model.py tests/test_gpu_atlas_shapes.py \
  tests/test_gpu_multi.py tests/test_gpu_batch.py > gpurun_out/r05m_tests.log 2>&1
step timeout -k 10 200 python -u tools/host_floor.py --sizes 2000 --iters 3 > gpurun_out/r05m_host_floor.txt 2>&1
step timeout -k 10 200 python -u tools/host_profile.py --N 2000 > gpurun_out/r05m_host_profile.txt 2>&1
echo done
