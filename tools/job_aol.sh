source tools/gpu_round.sh
export TAILN=4
step kern timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "apply_on_load or fused_bn_backward or normalise_on_load or wgrad"
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py tests/test_inference_gpu.py tests/test_trainer_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step benchA timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_AOL=0 step benchA_noaol timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_AOL=0 step benchC_noaol timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
