source tools/gpu_round.sh
export TAILN=4
step kern timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad"
python -c "
import json; p='mtl_das_pytorch_amd/engine/tuned_cfgs.json'; c=json.load(open(p))
json.dump({k: v for k, v in c.items() if not k.startswith('wgrad|')}, open(p, 'w'), indent=0, sort_keys=True)"
cp mtl_das_pytorch_amd/engine/tuned_cfgs.json gpurun_out/tuned_cfgs.json
step tuneA timeout -k 10 300 python bench.py --steps 50 --warmup 5
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
step tuneC timeout -k 10 300 python bench.py --model multi_classifier --steps 20 --warmup 5
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step benchA timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
