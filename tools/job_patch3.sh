source tools/gpu_round.sh
export TAILN=1
E=mtl_das_pytorch_amd/engine/tuned_cfgs.json
step new1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=64 step new_t64 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=256 step new_t256 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp $E /tmp/new.json
cp tools/cache_base.json $E
step base1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp /tmp/new.json $E
step new2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp tools/cache_base.json $E
step base2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp /tmp/new.json $E
step newC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_PATCH_TARGET=64 step newC_t64 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
