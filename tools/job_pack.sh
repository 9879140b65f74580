source tools/gpu_round.sh
export TAILN=4
step eng timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py -x -q --timeout 300 --timeout-method thread
export TAILN=1
step benchA timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step benchC timeout -k 10 300 python bench.py --model multi_classifier --steps 100 --warmup 10 --no-tune
cd /tmp && export TMPDIR=/tmp
step profC timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profC -o run -- python $GRAFT_REPO_ROOT/bench.py --model multi_classifier --steps 20 --warmup 5 --no-tune
