source tools/gpu_round.sh
export TAILN=3
step base timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-tune
export MDA_STREAMS=1
step ms timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-tune
step msdet timeout -k 10 300 python -m pytest tests/test_engine_gpu.py tests/test_inference_gpu.py -q -x -k "graph_replay or deterministic"
