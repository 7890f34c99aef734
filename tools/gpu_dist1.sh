# the N>1 launch path of bench.py with one rank (torch.distributed.run, nccl = RCCL)
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/dist1.log 2>&1
