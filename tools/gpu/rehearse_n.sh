# multi-rank rehearsal of the default bench on a 1-GPU box (gloo, every rank on cuda:0)
set -e
export PYTHONUNBUFFERED=1 DICP_BENCH_REHEARSE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err
