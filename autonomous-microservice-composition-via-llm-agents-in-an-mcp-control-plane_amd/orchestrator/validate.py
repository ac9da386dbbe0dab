"""T2 DAG validation and shape normalisation.

The reference never validates planner output (control_plane.py:74-75, SURVEY
D13) and its prompt asks for a different shape ("service_name, input_keys,
next_steps, fallback", control_plane.py:62) than ``/execute`` consumes (T2,
SURVEY D7).  ``normalize_dag`` converts that step-list shape into T2 and
``validate_dag`` checks a T2 graph (used by tests, the bench and the planner's
post-condition; ``/execute`` itself keeps the reference's permissive parsing).
"""
from __future__ import annotations

from typing import Iterable, Optional


class DagValidationError(ValueError):
    pass


def validate_dag(dag, registry_names: Optional[Iterable[str]] = None) -> None:
    if not isinstance(dag, dict):
        raise DagValidationError("DAG must be a JSON object")
    nodes, edges = dag.get("nodes"), dag.get("edges")
    if not isinstance(nodes, list) or not isinstance(edges, list):
        raise DagValidationError("DAG needs 'nodes' and 'edges' lists")
    names = []
    for n in nodes:
        if not isinstance(n, dict):
            raise DagValidationError("node must be an object")
        for k in ("name", "endpoint", "inputs"):
            if k not in n:
                raise DagValidationError(f"node missing '{k}'")
        if not isinstance(n["inputs"], dict):
            raise DagValidationError("node 'inputs' must be an object")
        names.append(n["name"])
    if len(set(names)) != len(names):
        raise DagValidationError("duplicate node names")
    known = set(names)
    if registry_names is not None:
        reg = set(registry_names)
        bad = [x for x in names if x not in reg]
        if bad:
            raise DagValidationError(f"unknown services {bad}")
    indeg = {x: 0 for x in names}
    adj = {x: [] for x in names}
    for e in edges:
        if not isinstance(e, dict) or "from" not in e or "to" not in e:
            raise DagValidationError("edge needs 'from' and 'to'")
        if e["from"] not in known or e["to"] not in known:
            raise DagValidationError("edge references unknown node")
        adj[e["from"]].append(e["to"])
        indeg[e["to"]] += 1
    ready = [x for x in names if indeg[x] == 0]
    seen = 0
    while ready:
        x = ready.pop()
        seen += 1
        for y in adj[x]:
            indeg[y] -= 1
            if indeg[y] == 0:
                ready.append(y)
    if seen != len(names):
        raise DagValidationError("DAG has a cycle")


def normalize_dag(dag, registry=None) -> dict:
    """Accept T2 as-is; convert the reference prompt's step-list shape to T2."""
    if isinstance(dag, dict) and "nodes" in dag:
        dag.setdefault("edges", [])
        return dag
    steps = dag.get("steps") if isinstance(dag, dict) else dag
    if not isinstance(steps, list):
        raise DagValidationError("unrecognised DAG shape")
    nodes, edges = [], []
    for s in steps:
        name = s.get("service_name") or s.get("name")
        rec = registry.get(name) if registry is not None else None
        endpoint = s.get("endpoint") or (rec.endpoint if rec is not None else None)
        keys = s.get("input_keys") or []
        nodes.append({"name": name, "endpoint": endpoint, "inputs": {k: k for k in keys}})
        for nxt in s.get("next_steps") or []:
            e = {"from": name, "to": nxt}
            if s.get("fallback"):
                e["fallback"] = s["fallback"]
            edges.append(e)
    return {"nodes": nodes, "edges": edges}
