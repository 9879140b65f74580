source tools/gpu_round.sh
export TAILN=15
step infgpu timeout -k 10 600 python -m pytest tests/test_inference_gpu.py -x -q
