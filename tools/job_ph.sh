source tools/gpu_round.sh
export TAILN=8
step phA timeout -k 10 240 python tools/phase_times.py MTL 300
MDA_STREAMS=0 step phA_serial timeout -k 10 240 python tools/phase_times.py MTL 300
step phC timeout -k 10 300 python tools/phase_times.py multi_classifier 100
step benchA timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-tune
