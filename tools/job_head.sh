source tools/gpu_round.sh
export TAILN=3
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inference_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step bench timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchB timeout -k 10 200 python bench.py --model single_event --steps 400 --warmup 30 --no-tune
export TAILN=4
step lt timeout -k 10 300 python tools/launch_times.py MTL fwd
