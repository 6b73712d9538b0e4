# round 5: adaptive re-referencing after one tile -- E-step against sigma, A/B line, and the
# bench's own E-step under rocprofv3 (kernel stats)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05v
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
step timeout -k 10 200 python -u tools/probes/estep_sigma.py > gpurun_out/r05v_estep_sigma.jsonl 2> gpurun_out/r05v.err
step timeout -k 10 300 python -u tools/ab_libs.py --M 100000 --passes 2 base > gpurun_out/r05v_ab.json 2>> gpurun_out/r05v.err
cd /tmp && export TMPDIR=/tmp
step timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05v/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05v/bench.log 2>&1
echo done
