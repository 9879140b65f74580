source tools/gpu_round.sh
export TAILN=6
export MDA_SINGLE_DEVICE=1 MDA_DIST_BACKEND=gloo
step dp2 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 30 --warmup 5
step dp2C timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 2 --steps 10 --warmup 3 --model multi_classifier
