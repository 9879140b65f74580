source tools/gpu_round.sh
export TAILN=2
step ltC timeout -k 10 400 python tools/launch_times.py multi_classifier bwd
MDA_DGRAD_BNSTATS=0 step ltC_nobns timeout -k 10 400 python tools/launch_times.py multi_classifier bwd
step ltCf timeout -k 10 400 python tools/launch_times.py multi_classifier fwd
