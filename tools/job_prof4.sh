source tools/gpu_round.sh
export TAILN=3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step profA timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profA4 -o run -- python3 bench.py --steps 30 --warmup 3 --no-tune
step profC timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profC4 -o run -- python3 bench.py --model multi_classifier --steps 20 --warmup 3 --no-tune
