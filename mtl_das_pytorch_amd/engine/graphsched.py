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
joins) and runs the executor's assignment on it, so that an issue order (Phase.ISSUE_ORDER) can be chosen
on the CPU that makes the executor's streams coincide with the engine's logical streams."""
from __future__ import annotations

import re
import sys
from typing import Dict, List, Sequence

from .program import Phase, stream_slots

import os  # noqa: E402

# the executor's stream count (DEBUG_HIP_FORCE_GRAPH_QUEUES: runtime default 4, the package sets 2)
EXEC_STREAMS = int(os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES", "4"))


def launch_records(phases: Sequence[Phase]) -> List[dict]:
    """The launches of ``phases`` in host issue order, as plain records: phase index, name, physical stream
    slot (program.stream_slots), waits (resolved through the phase's aliases), recorded tag, and whether the
    launch issues a kernel."""
    out = []
    for pi, ph in enumerate(phases):
        slot = stream_slots(ph.launches)
        for l in ph.issue_order():
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


def schedule(children: List[List[int]], n_streams: int = EXEC_STREAMS) -> List[int]:
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


def mismatch(phases: Sequence[Phase], n_streams: int = EXEC_STREAMS) -> dict:
    """How far the executor's assignment is from the logical one: for every logical stream, the executor
    streams its kernels land on (count per stream), and the number of kernels not on the executor stream
    that holds most of their logical stream."""
    nodes, children = capture_dag(launch_records(phases))
    sid = schedule(children, n_streams)
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


def plan_children(children: List[List[int]], target: List, n_streams: int = EXEC_STREAMS):
    """New per-node child orders (with redundant filler edges) under which the executor's assignment
    (``schedule``) puts every node whose ``target`` is known on exactly that executor stream.

    Why it works: a node's first child inherits its stream, the child at edge position p gets stream + p.
    * position 0 of every node is its same-target successor (the next node of its logical stream), so
      the walk from the root first dives down the whole stream-0 chain, then each chain is followed down
      from wherever it is first entered;
    * a child on another non-zero target is placed at a position p = (its target - the node's) mod
      n_streams, so that it is right whichever of its parents reaches it first;
    * children that are already scheduled when the node's loop reaches them -- stream-0 nodes (scheduled by
      the initial dive) and later nodes of the node's own chain (scheduled by its position-0 dive) -- fill
      the gaps; when they run out, redundant edges to such nodes are added (the node already precedes
      them, so no dependency changes).
    Nodes with an unknown target (None) keep their child order.  Returns (new children, #filler edges)."""
    n = len(children)
    N = n_streams
    parents = [[] for _ in range(n)]
    for v, cs in enumerate(children):
        for c in cs:
            parents[c].append(v)

    def succ(v):
        if target[v] is None:
            return None
        return next((c for c in children[v] if target[c] == target[v]), None)

    nxt = [succ(v) for v in range(n)]
    new, fillers = [], 0
    for v in range(n):
        cs = children[v]
        tv = target[v]
        if tv is None or not cs:
            new.append(list(cs))
            continue
        s = nxt[v]
        constrained = {}
        free = []
        for c in cs:
            if c == s:
                continue
            tc = target[c]
            if tc is None or tc == 0 or tc == tv:
                free.append(c)
            else:
                constrained.setdefault((tc - tv) % N, []).append(c)
        # spare filler nodes: the node's own chain below its successor, then stream-0 descendants
        have = set(cs)
        spare = []

        def more_spare():
            if spare:
                return spare.pop(0)
            return None

        chain, x = [], (nxt[s] if s is not None else None)
        while x is not None and len(chain) < 3 * N:
            if x not in have:
                chain.append(x)
            x = nxt[x]
        spare.extend(chain)
        out = [s] if s is not None else []
        if s is None and constrained:  # position 0 must not take a constrained child
            f = free.pop(0) if free else more_spare()
            if f is None:
                new.append(list(cs))
                continue
            if f not in have:
                fillers += 1
            out.append(f)
        ok = True
        while any(constrained.values()):
            r = len(out) % N
            if constrained.get(r):
                out.append(constrained[r].pop(0))
                continue
            f = free.pop(0) if free else more_spare()
            if f is None:
                ok = False
                break
            if f not in have:
                fillers += 1
                have.add(f)
            out.append(f)
        if not ok:
            new.append(list(cs))
            continue
        out += free
        new.append(out)
    return new, fillers


def restream_check(children: List[List[int]], target: List, n_streams: int = EXEC_STREAMS):
    """(#nodes with a known target, #of them the executor would put elsewhere) for a child order."""
    sid = schedule(children, n_streams)
    known = [i for i, t in enumerate(target) if t is not None]
    return len(known), sum(1 for i in known if sid[i] != target[i])


def restream(graph: int, tracker) -> dict:
    """Rewrite the edge order of a captured (not yet instantiated) graph so that the executor runs every
    tracked node on the executor stream of its engine stream (plan_children).  Applied only when the
    emulated assignment is then exact; returns what was done."""
    from ..ops.hip import lib
    _, children = lib().graph_structure(graph)
    # more engine streams than executor streams: stream 0 keeps an executor stream of its own, the side
    # streams fold onto the others
    targets = [None if t is None else min(t, EXEC_STREAMS - 1) for t in tracker.targets(graph)]
    known, before = restream_check(children, targets)
    new, fillers = plan_children(children, targets)
    _, after = restream_check(new, targets)
    applied = after < before
    if applied:
        lib().graph_set_children(graph, new)
    return {"nodes": len(children), "tracked": known, "misplaced_before": before, "misplaced_after": after,
            "fillers": fillers, "applied": applied}
