"""What the HIP graph executor does with a captured multi-stream step, emulated on the host.

A stream capture records a DAG, not streams: when ``hipGraphLaunch`` runs the executable, the runtime
re-derives its own stream per node (``DEBUG_HIP_GRAPH_DOT_PRINT=1`` prints them as ``StreamId``).
Measured on MI355X / ROCm 7 (tools/graph_dot.py; the emulation below reproduces every node's StreamId of the
captured Model A and C steps): a depth-first walk from the root nodes (roots get executor streams 0, 1, 2, ...
in creation order), where the child at edge position p of a node (edge insertion order, counting every
edge) gets the node's stream + p modulo the executor's stream count (4), unless an earlier part of the
walk already scheduled it.  Executor stream 0 is the
launch stream; the others are streams the executable created.  So the logical streams the engine captured
on are NOT what runs: e.g. Model A's captured backbone (logical stream 0) ran split over two queues, the
level branches over the same two (tools/timeline.py queue column).

This module rebuilds the DAG a capture of engine phases produces (the capture semantics of
``Phase.run``: per-stream dependency sets, event records / waits, the phase-start fork and phase-end
joins) and runs the executor's assignment on it: an analysis tool (tools/graph_dot.py, profiles/
r5_graph_streams.md).  Rewriting a captured graph's edge order so that the executor keeps every engine stream
on a stream of its own was built in round 5 and measured SLOWER (A -1.7 %, C -7 %: more kernels compete for
the CUs at once); it was removed, the measurement is in docs/PERF.md.  The engine instead runs with 2 executor
streams (DEBUG_HIP_FORCE_GRAPH_QUEUES, set by the entry points: mtl_das_pytorch_amd.use_engine_graph_queues)."""
from __future__ import annotations

import re
import sys
from typing import Dict, List, Sequence

from .program import Phase, stream_slots

import os  # noqa: E402


def executor_streams() -> int:
    """The executor's stream count as the environment requests it (DEBUG_HIP_FORCE_GRAPH_QUEUES, runtime default
    4; the entry points set 2).  The runtime reads the variable once, at its initialisation: a value set after
    the process's first HIP call is not the one in effect."""
    return int(os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES", "4"))


def launch_records(phases: Sequence[Phase]) -> List[dict]:
    """The launches of ``phases`` in host issue order, as plain records: phase index, name, physical stream
    slot (program.stream_slots), waits (resolved through the phase's aliases), recorded tag, and whether the
    launch issues a kernel."""
    out = []
    for pi, ph in enumerate(phases):
        slot = stream_slots(ph.launches)
        for l in ph.launches:
            out.append({"phase": pi, "name": l.name, "stream": slot[l.stream], "logical": l.stream,
                        "waits": [f"{pi}:{ph.alias.get(t, t)}" for t in l.waits],
                        "record": None if l.record is None else f"{pi}:{l.record}", "kernel": l.fn is not None})
    return out


def capture_dag(records: List[dict]):
    """The DAG a stream capture of ``records`` builds.  Returns (nodes, children): nodes[i] is the record
    of node i (nodes in creation order), children[i] the child nodes of i in edge-insertion order."""
    last: Dict[int, List[int]] = {0: []}  # per physical stream: the nodes its next node depends on
    events: Dict[str, List[int]] = {}
    nodes, children = [], []
    phase = None
    used: set = set()

    def join():
        for s in used - {0}:  # main.wait_stream(side)
            last[0] = list(dict.fromkeys(last[0] + last.get(s, [])))

    for r in records:
        if r["phase"] != phase:
            if phase is not None:
                join()
            phase = r["phase"]
            used = {x["stream"] for x in records if x["phase"] == phase}
            for s in used - {0}:  # every side stream waits for the phase-start event recorded on stream 0
                last[s] = list(last[0])
        s = r["stream"]
        deps = list(last.get(s, []))
        for t in r["waits"]:
            deps = list(dict.fromkeys(deps + events[t]))
        if r["kernel"]:
            v = len(nodes)
            nodes.append(r)
            children.append([])
            for d in deps:
                children[d].append(v)
            last[s] = [v]
        else:
            last[s] = deps
        if r["record"] is not None:
            events[r["record"]] = list(last[s])
    return nodes, children


def schedule(children: List[List[int]], n_streams: int = 4) -> List[int]:
    """The executor's stream per node (see the module docstring)."""
    n = len(children)
    indeg = [0] * n
    for cs in children:
        for c in cs:
            indeg[c] += 1
    sid = [-1] * n
    limit = sys.getrecursionlimit()
    sys.setrecursionlimit(max(limit, 10 * n + 1000))

    def one(v, s):
        sid[v] = s
        for c in children[v]:  # the stream advances for EVERY edge, scheduled child or not
            if sid[c] == -1:
                one(c, s)
            s = (s + 1) % n_streams

    try:
        r = 0
        for v in range(n):
            if indeg[v] == 0 and sid[v] == -1:
                one(v, r)
                r = (r + 1) % n_streams
    finally:
        sys.setrecursionlimit(limit)
    return sid


def mismatch(phases: Sequence[Phase], n_streams: int = None) -> dict:
    """How far the executor's assignment is from the logical one: for every logical stream, the executor
    streams its kernels land on (count per stream), and the number of kernels not on the executor stream
    that holds most of their logical stream."""
    nodes, children = capture_dag(launch_records(phases))
    sid = schedule(children, executor_streams() if n_streams is None else n_streams)
    per: Dict[int, Dict[int, int]] = {}
    for r, s in zip(nodes, sid):
        per.setdefault(r["stream"], {}).setdefault(s, 0)
        per[r["stream"]][s] += 1
    off = sum(sum(d.values()) - max(d.values()) for d in per.values())
    shared = len(per) - len({max(d, key=d.get) for d in per.values()})
    return {"per_stream": per, "off": off, "shared_home": shared}


def parse_dot(path: str):
    """Nodes (kernel name, StreamId) and edges (insertion order) of a DEBUG_HIP_GRAPH_DOT_PRINT dump."""
    txt = open(path).read()
    nodes = {}
    for m in re.finditer(r'"graph_\d+_node_(\d+)"\[[^\]]*label="\d+\n([^\n]*)\nStreamId:(-?\d+)', txt):
        nodes[int(m.group(1))] = (m.group(2), int(m.group(3)))
    edges = [(int(a), int(b)) for a, b in re.findall(r'"graph_\d+_node_(\d+)" -> "graph_\d+_node_(\d+)"', txt)]
    n = max(nodes) + 1 if nodes else 0
    children = [[] for _ in range(n)]
    for a, b in edges:
        children[a].append(b)
    return [nodes[i] for i in range(n)], children
