source tools/gpu_round.sh
export TAILN=25
step incep timeout -k 10 600 python -m pytest tests/test_inception_gpu.py -q -s
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 30 --warmup 5 --no-tune
