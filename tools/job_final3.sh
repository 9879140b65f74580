source tools/gpu_round.sh
export TAILN=4
step gpu timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
export TAILN=1
step benchdef timeout -k 10 400 python bench.py
