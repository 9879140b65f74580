source tools/gpu_round.sh
export TAILN=8
step gputests timeout -k 10 900 python -m pytest tests -m gpu -x -q
rm -f gpurun_out/tuned_cfgs.json
step benchA timeout -k 10 300 python bench.py --steps 200 --warmup 20
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json || true
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10
