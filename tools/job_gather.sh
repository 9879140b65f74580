source tools/gpu_round.sh
export TAILN=3
step t timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "gather or stem or autograd"
export TAILN=1
step a1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step a2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
export TAILN=6
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
