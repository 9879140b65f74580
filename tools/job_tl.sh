source tools/gpu_round.sh
export TAILN=2
step tlA timeout -k 10 200 python tools/timeline.py MTL
step tlC timeout -k 10 300 python tools/timeline.py multi_classifier
