source tools/gpu_round.sh
export TAILN=2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step pmcC timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE SQ_WAVES --output-format csv -d gpurun_out/pmcC -o run -- python3 bench.py --model multi_classifier --steps 5 --warmup 2 --no-tune
