source tools/gpu_round.sh
export TAILN=2
step tlA timeout -k 10 200 python tools/timeline.py MTL
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
