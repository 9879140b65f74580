source tools/gpu_round.sh
export TAILN=3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step profA timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profA3 -o run -- python3 bench.py --steps 30 --warmup 3 --no-tune
step profC timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profC3 -o run -- python3 bench.py --model multi_classifier --steps 20 --warmup 3 --no-tune
step ltA timeout -k 10 300 python tools/launch_times.py MTL bwd
