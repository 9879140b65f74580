source tools/gpu_round.sh
export TAILN=4
for i in 1 2 3; do
timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -q -s -k graph_replay 2>&1 | grep -E "one-step|passed|failed" 
done
