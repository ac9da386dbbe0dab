"""Plan auditing: human-readable explanations and telemetry-adaptive plans.

The reference README claims both (``README.md:43-44`` "real-time metrics ...
enabling adaptive planning", ``README.md:48`` "incorporates live telemetry",
``README.md:50`` "human-readable explanations for auditability") but
``control_plane.py`` implements neither.  Here:

* ``explain_plan(graph, registry)`` renders a deterministic audit text for a
  DAG (T2): execution order by topological generation (T3, the order the
  orchestrator runs and the ``results`` keys follow), where each input comes
  from (an upstream node's whole body or a payload field, T4), retries and the
  ordered fallback chain the orchestrator would try, the registry's
  ``cost_profile`` and observed telemetry, and the plan's total cost.
* ``adapt_plan(graph, registry)`` is the adaptive step.  Telemetry changes on
  every call, so it is applied to the planner's output rather than fed into
  the prompt: putting it in the prompt would invalidate the cached registry
  prefix (and its KV blocks) on every request.  A node whose service shows an
  error rate at or above a threshold gets extra retries and the registry
  record's fallback appended to its ordered ``fallbacks`` list (node keys the
  orchestrator already honours), so the DAG stays in the T2 shape.
* ``AdaptivePlanner`` wraps any planner with ``adapt_plan``
  (``MCP_ADAPTIVE=1``).
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

from .base import Planner


def _generations(graph: dict) -> List[List[str]]:
    from ..orchestrator.executor import Orchestrator
    return Orchestrator.generations(Orchestrator.build_graph(graph))


def _telemetry(registry, name: str) -> Dict[str, float]:
    if registry is None:
        return {}
    try:
        return registry.telemetry(name) or {}
    except Exception:          # telemetry is advisory; a registry error must not fail a plan
        return {}


def _rates(tel: Dict[str, float]):
    calls = float(tel.get("calls", 0) or 0)
    if calls <= 0:
        return 0, None, None
    return int(calls), float(tel.get("errors", 0) or 0) / calls, \
        float(tel.get("latency_sum", 0.0) or 0.0) / calls


def fallback_chain(graph: dict, name: str, registry=None,
                   use_registry_fallback: bool = False) -> List[str]:
    """The fallback URLs the orchestrator tries for ``name``, in order
    (first in-edge, node ``fallbacks``, node ``fallback``, registry)."""
    out: List[str] = []
    for e in graph.get("edges", []):
        if e.get("to") == name:
            if e.get("fallback"):
                out.append(e["fallback"])
            break
    node = next((n for n in graph["nodes"] if n.get("name") == name), {})
    if isinstance(node.get("fallbacks"), list):
        out += [f for f in node["fallbacks"] if isinstance(f, str) and f]
    if isinstance(node.get("fallback"), str) and node["fallback"]:
        out.append(node["fallback"])
    if use_registry_fallback and registry is not None:
        rec = registry.get(name)
        if rec is not None and rec.get("fallback"):
            out.append(rec["fallback"])
    return list(dict.fromkeys(out))


def explain_plan(graph: dict, registry=None, default_retries: int = 0,
                 use_registry_fallback: bool = False) -> str:
    """Deterministic, human-readable account of what executing ``graph`` does.
    Raises like the orchestrator on a malformed DAG (missing ``edges``,
    cycle), so an explanation is only produced for a plan that would run."""
    gens = _generations(graph)
    nodes = {n["name"]: n for n in graph["nodes"]}
    produced = set()
    lines = [f"Plan with {len(nodes)} step(s) in {len(gens)} stage(s)."]
    total_cost, priced = 0.0, 0
    step = 0
    for g, names in enumerate(gens):
        par = " (independent steps, may run concurrently)" if len(names) > 1 else ""
        lines.append(f"Stage {g + 1}{par}:")
        for name in names:
            step += 1
            node = nodes.get(name, {})
            lines.append(f"  {step}. {name} -> POST {node.get('endpoint', '?')}")
            ins = node.get("inputs") or {}
            if not ins:
                lines.append("     inputs: none")
            for k, src in ins.items():
                if src in nodes:
                    how = f"the full response of step '{src}'"
                    if src not in produced:
                        how += " (not yet produced: falls back to the payload)"
                else:
                    how = f"payload field '{src}' (null when absent)"
                lines.append(f"     input '{k}' <- {how}")
            retries = node.get("retries", default_retries)
            chain = fallback_chain(graph, name, registry, use_registry_fallback)
            fail = (f"on failure: {retries} retr{'y' if retries == 1 else 'ies'}, then "
                    if isinstance(retries, int) and retries > 0 else "on failure: ")
            if chain:
                fail += "fallbacks in order: " + ", ".join(chain)
            else:
                fail += "no fallback, the whole request aborts with HTTP 502"
            lines.append(f"     {fail}")
            rec = registry.get(name) if registry is not None else None
            if rec is not None and isinstance(rec.get("cost_profile"), (int, float)):
                total_cost += float(rec["cost_profile"])
                priced += 1
                lines.append(f"     cost profile: {rec['cost_profile']}")
            calls, err, lat = _rates(_telemetry(registry, name))
            if calls:
                lines.append(f"     telemetry: {calls} call(s), error rate {err:.1%}, "
                             f"mean latency {lat * 1e3:.1f} ms")
            produced.add(name)
    if priced:
        lines.append(f"Estimated cost: {total_cost:.6g} ({priced} of {len(nodes)} step(s) priced).")
    return "\n".join(lines)


def adapt_plan(graph: dict, registry, error_rate: float = 0.2, min_calls: int = 5,
               retries: int = 1) -> dict:
    """Telemetry-adaptive hardening of a plan (a copy is returned).  Nodes whose
    service has ``>= min_calls`` recorded calls and an error rate
    ``>= error_rate`` get ``retries`` (at least) and the registry record's
    fallback appended to ``fallbacks``; each change is listed in the node's
    ``adapted`` attribute for auditing."""
    out = copy.deepcopy(graph)
    if registry is None:
        return out
    for node in out.get("nodes", []):
        name = node.get("name")
        calls, err, _ = _rates(_telemetry(registry, name))
        if calls < max(1, min_calls) or err is None or err < error_rate:
            continue
        why = []
        cur = node.get("retries")
        if not isinstance(cur, int) or cur < retries:
            node["retries"] = retries
            why.append(f"retries={retries}")
        rec = registry.get(name)
        fb = rec.get("fallback") if rec is not None else None
        if fb:
            lst = node.get("fallbacks") if isinstance(node.get("fallbacks"), list) else []
            if fb not in lst and fb != node.get("fallback"):
                node["fallbacks"] = lst + [fb]
                why.append(f"fallback {fb}")
        if why:
            node["adapted"] = f"error rate {err:.1%} over {calls} calls: " + ", ".join(why)
    return out


class AdaptivePlanner(Planner):
    """Applies ``adapt_plan`` to every plan of the wrapped planner."""

    def __init__(self, inner: Planner, registry, error_rate: float = 0.2,
                 min_calls: int = 5, retries: int = 1):
        self.inner = inner
        self.registry = registry
        self.error_rate = error_rate
        self.min_calls = min_calls
        self.retries = retries

    async def plan(self, intent: str) -> dict:
        dag = await self.inner.plan(intent)
        if not isinstance(dag, dict) or not isinstance(dag.get("nodes"), list):
            return dag         # malformed output keeps the reference's error path
        return adapt_plan(dag, self.registry, self.error_rate, self.min_calls, self.retries)

    async def aclose(self):
        await self.inner.aclose()

    def __getattr__(self, name):
        return getattr(self.inner, name)


__all__ = ["explain_plan", "adapt_plan", "fallback_chain", "AdaptivePlanner"]
