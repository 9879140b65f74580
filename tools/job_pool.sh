source tools/gpu_round.sh
export TAILN=3
step t timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_inception_gpu.py -x -q --timeout 300 --timeout-method thread -k "pool or inception"
export TAILN=1
step C timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_POOL_ARGMAX=0 step Cno timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
step C2 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_POOL_ARGMAX=0 step Cno2 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
