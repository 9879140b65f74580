source tools/gpu_round.sh
export TAILN=1
for i in 1 2; do
step A_base_$i timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
MDA_PRIO=1 step A_prio_$i timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-tune
done
