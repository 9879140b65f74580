source tools/gpu_round.sh
export TAILN=1
step m3 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAXB=99 step m99 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAXB=2 step m2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAXB=4 step m4 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAXB=1 step m1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step m3b timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step C3 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_WGRAD_MAXB=99 step C99 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_WGRAD_MAXB=2 step C2 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
