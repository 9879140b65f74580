source tools/gpu_round.sh
export TAILN=2
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inference_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step A1 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step A2 timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step B timeout -k 10 200 python bench.py --model single_event --steps 400 --warmup 30 --no-tune
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
step tlA timeout -k 10 200 python tools/timeline.py MTL
