source tools/gpu_round.sh
export TAILN=4
step kern timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py tests/test_inference_gpu.py -x -q --timeout 300 --timeout-method thread
step tuneA timeout -k 10 300 python bench.py --steps 50 --warmup 5
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
step tuneC timeout -k 10 300 python bench.py --model multi_classifier --steps 20 --warmup 5
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
step phC timeout -k 10 300 python tools/phase_times.py multi_classifier 100
step benchA timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
