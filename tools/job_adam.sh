source tools/gpu_round.sh
export TAILN=3
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inference_gpu.py tests/test_inception_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step bench timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_FUSED_ADAM=0 step bench_unf timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_FUSED_ADAM=0 step benchC_unf timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
step bench2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
export TAILN=6
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
