# round 5: the eta != 0 VJP's unwritten-workspace reads (slot probe, poison probe), the graph and
# EM tests on the fixed dead-component logit, the atlas rehearsals at W = 4 / 8 (graphs blocked
# under concurrent frames), then the PMC passes.  A pytest FAILURE (rc 1) is recorded and the
# script goes on; any other status stops it.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
tstep() { "$@"; rc=$?; case $rc in 0|1) echo "tests rc=$rc"; return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
step timeout -k 10 200 python -u tools/probes/eta_slots.py > gpurun_out/r05j_eta_slots.jsonl 2> gpurun_out/r05j_eta_slots.err
tstep timeout -k 10 300 $T tests/test_gpu_em.py tests/test_gpu_shoot_graph.py > gpurun_out/r05j_tests.log 2>&1
export DICP_BENCH_REHEARSE=1
for W in 4 8; do
  step timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 \
    --master-port 2953$W bench.py --gpus $W --workload atlas_c4_fixed --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_rehearsal_atlas_c4_fixed_w$W.json 2> gpurun_out/r05_rehearsal_atlas_c4_fixed_w$W.err
done
unset DICP_BENCH_REHEARSE
step bash tools/gpu/r05_pmc.sh
echo done
