source tools/gpu_round.sh
export TAILN=3
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py tests/test_inference_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step split timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_FIN_SPLIT=0 step nosplit timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step split2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_FIN_SPLIT=0 step nosplit2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step C timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_FIN_SPLIT=0 step Cno timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
