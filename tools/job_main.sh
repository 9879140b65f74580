source tools/gpu_round.sh
export TAILN=3
step adamt timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "adam or batched"
export TAILN=1
step base timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAIN=1 step main3 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAIN=1 MDA_WGRAD_MAXB=4 step main4 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAIN=1 MDA_WGRAD_MAXB=2 step main2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step base2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAIN=1 step main3b timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
