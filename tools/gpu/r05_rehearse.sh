# round 5: multi-rank rehearsals of the bench on a 1-GPU box -- every rank
# on cuda:0 over gloo (DICP_BENCH_REHEARSE=1, the line's parallelism says so): the row-split
# two-set match at W = 4 (the overlapped two-phase steps switch on from W = 4) and W = 8, and
# the fixed 32-frame C4 atlas at W = 4 and 8 (frame sharding, one statistics exchange per EM step)
export PYTHONUNBUFFERED=1 DICP_BENCH_REHEARSE=1
mkdir -p gpurun_out
step() { "$@"; rc=$?; case $rc in 0) return 0;; *) echo "step rc=$rc: stopping"; exit $rc;; esac; }
run() {   # W workload port
  step timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $3 bench.py --gpus $1 --workload $2 --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_rehearsal_$2_w$1.json 2> gpurun_out/r05_rehearsal_$2_w$1.err
}
run 4 two_set_100k 29521
run 8 two_set_100k 29522
run 4 atlas_c4_fixed 29523
run 8 atlas_c4_fixed 29524
