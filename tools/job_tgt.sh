source tools/gpu_round.sh
export TAILN=1
step t128 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=64 step t64 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=256 step t256 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=32 step t32 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step t128b timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_WGRAD_MAXB=2 MDA_PATCH_TARGET=64 step m2t64 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
