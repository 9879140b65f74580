source tools/gpu_round.sh
export TAILN=4
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step profA timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profA4 -o run -- python3 bench.py --steps 30 --warmup 3 --no-tune
