source tools/gpu_round.sh
export TAILN=1
step C1024 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_MIN_SPLIT_PX=2048 step C2048 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_MIN_SPLIT_PX=4096 step C4096 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
step A1024 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_MIN_SPLIT_PX=2048 step A2048 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_MIN_SPLIT_PX=512 step A512 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
