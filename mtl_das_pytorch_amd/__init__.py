"""mtl_das_pytorch_amd: MI355X-native multi-task DAS training framework."""
import os as _os

__version__ = "0.1.0"

# The HIP graph executor re-derives the streams of a captured step itself and spreads it over
# DEBUG_HIP_FORCE_GRAPH_QUEUES streams (runtime default 4; engine/graphsched.py).  The engine's step is
# latency-bound and its critical chain loses more to concurrent side branches than the branches gain:
# with 2 executor streams Model C trains 9.01 / 9.03 k samples/s against 8.29 / 8.26 k with 4 (3: 8.43 / 8.52 k,
# 5 and 8: 8.21 / 8.18 k), Model A 35.40 k against 35.39 k (docs/PERF.md round 5).  The runtime reads it when it
# initialises, so it is set here, before the first HIP call of the process; an explicit setting wins.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")
