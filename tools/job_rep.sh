source tools/gpu_round.sh
export TAILN=1
for i in 1 2; do
step A_nol_$i timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_NOL=0 step A_off_$i timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
step C_nol_$i timeout -k 10 300 python bench.py --model multi_classifier --steps 150 --warmup 10 --no-tune
MDA_NOL=0 step C_off_$i timeout -k 10 300 python bench.py --model multi_classifier --steps 150 --warmup 10 --no-tune
done
