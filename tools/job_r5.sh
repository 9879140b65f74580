source tools/gpu_round.sh
export TAILN=8
step race timeout -k 10 250 python tools/dbg_race.py
for i in 1 2; do timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -q -s -k graph_replay 2>&1 | grep -E "one-step|passed|failed"; done
step gputests timeout -k 10 900 python -m pytest tests -m gpu -x -q
rm -f gpurun_out/tuned_cfgs.json
step benchA timeout -k 10 300 python bench.py --steps 200 --warmup 20
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json || true
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10
