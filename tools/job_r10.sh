source tools/gpu_round.sh
export TAILN=8
step gputests timeout -k 10 900 python -m pytest tests -m gpu -x -q
step benchA timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
