source tools/gpu_round.sh
export TAILN=1
step kern timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread
step eng timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k "autograd or bitwise or graph" --timeout 300 --timeout-method thread
for L in 16 4 1; do
  MDA_FIN_LANES=$L step lanes_$L timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
done
MDA_FIN_LANES=16 step benchC16 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
MDA_FIN_LANES=1 step benchC1 timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
