"""mtl_das_pytorch_amd: MI355X-native multi-task DAS training framework."""
import os as _os

__version__ = "0.1.0"

# The HIP graph executor re-derives the streams of a captured step itself and spreads it over
# DEBUG_HIP_FORCE_GRAPH_QUEUES streams (runtime default 4).  The engine's step is latency-bound and its critical
# chain loses more to concurrent side branches than the branches gain: with 2 executor streams Model C trains
# 9.01 / 9.03 k samples/s against 8.29 / 8.26 k with 4 (3: 8.43 / 8.52 k, 5 and 8: 8.21 / 8.18 k), Model A
# 35.40 k against 35.39 k (docs/PERF.md round 5).  The runtime reads the variable once, when it initialises, and
# it applies to every HIP graph of the process -- so importing the package does NOT set it (a host application's
# own graphs keep the runtime default); the entry points (bench.py, train.py, test.py, infer.py) call
# ``use_engine_graph_queues()`` before their first HIP call, and bench.py records the value in its JSON line.
GRAPH_QUEUES = "2"


def use_engine_graph_queues() -> str:
    """Select the engine's HIP graph executor stream count for this process unless the environment already sets
    one; returns the value in effect.  Only effective before the process's first HIP call."""
    return _os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", GRAPH_QUEUES)
