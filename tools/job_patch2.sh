source tools/gpu_round.sh
export TAILN=1
E=mtl_das_pytorch_amd/engine/tuned_cfgs.json
cp $E /tmp/orig.json
step base timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp tools/cache_p1.json $E
step p1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=128 step p1_t128 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
cp tools/cache_p2.json $E
step p2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PATCH_TARGET=128 step p2_t128 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step p2C timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_PATCH_TARGET=128 step p2C_t128 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
cp /tmp/orig.json $E
step baseC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
