source tools/gpu_round.sh
export TAILN=6
step eagerC timeout -k 10 300 python tools/eager_baseline.py --model multi_classifier
step eagerB timeout -k 10 300 python tools/eager_baseline.py --model single_event
step benchCtune timeout -k 10 600 python bench.py --model multi_classifier --steps 100 --warmup 10
cp gpurun_out/tuned_cfgs.json mtl_das_pytorch_amd/engine/tuned_cfgs.json
step benchB timeout -k 10 300 python bench.py --model single_event --steps 100 --warmup 10
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step profC timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profC -o run -- python3 bench.py --model multi_classifier --steps 20 --warmup 3 --no-tune
