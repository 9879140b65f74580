source tools/gpu_round.sh
export TAILN=6
step gpu timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TAILN=2
step profA timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profA5 -o run -- python3 bench.py --steps 30 --warmup 3 --no-tune
step tlA timeout -k 10 200 python tools/timeline.py MTL
