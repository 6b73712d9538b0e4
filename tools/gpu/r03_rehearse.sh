# round 3: multi-rank rehearsal on a 1-GPU box (gloo, every rank on cuda:0) of the default
# bench (two-set 100k row split) and of the fixed 32-frame atlas (frames sharded over ranks)
set -e
export PYTHONUNBUFFERED=1 DICP_BENCH_REHEARSE=1
mkdir -p gpurun_out/r03m
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03m/two_set2.json 2> gpurun_out/r03m/two_set2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload atlas_c4_fixed --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03m/c4fixed2.json 2> gpurun_out/r03m/c4fixed2.err
echo done
