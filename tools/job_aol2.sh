source tools/gpu_round.sh
export TAILN=4
step eng timeout -k 10 300 python -u -m pytest tests/test_inception_gpu.py -x -q --timeout 300 --timeout-method thread -k layer_local
export TAILN=1
step benchA timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_AOL=pw step benchA_pw timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_AOL=pw step benchC_pw timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
