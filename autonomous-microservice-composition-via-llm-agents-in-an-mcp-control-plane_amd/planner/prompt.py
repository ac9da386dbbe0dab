"""Planner prompt construction.

Reference prompt (control_plane.py:58-67): fixed instruction text, one line per
registry service (name, endpoint, input/output schema rendered as Python repr),
the intent in curly quotes, then ``JSON DAG:``.  Two reference defects are
fixed here: the instruction asks for the T2 shape that
``/execute`` actually consumes, and the text uses real newlines and JSON.

The prompt is split into a **registry prefix** (instructions + service list,
identical for every intent against the same registry version) and a per-intent
**suffix**.  The engine tokenises them separately and shares the prefix's KV
blocks between concurrent requests (prefix caching).
"""
from __future__ import annotations

import json
from typing import List, Sequence, Tuple

HEADER = (
    "You are the planning agent of a microservice control plane. Compose the "
    "available services into an execution graph that fulfils the user's intent.\n"
    "Answer with one JSON object and nothing else: {\"nodes\": [{\"name\": <service>, "
    "\"endpoint\": <url>, \"inputs\": {<input field>: <payload field or upstream node>}, "
    "\"retries\": <int>}], \"edges\": [{\"from\": <node>, \"to\": <node>, "
    "\"fallback\": <url>}]}. Edges must point from producers to consumers.\n\n"
    "Available services:\n"
)
# the grammar's compact model view (planner/grammar.py): endpoints and fallback
# URLs come from the registry, the model names services and marks fallbacks
HEADER_COMPACT = (
    "You are the planning agent of a microservice control plane. Compose the "
    "available services into an execution graph that fulfils the user's intent.\n"
    "Answer with one JSON object and nothing else: {\"nodes\": [{\"name\": <service>, "
    "\"inputs\": {<input field>: <payload field or upstream node>}, "
    "\"retries\": <int>}], \"edges\": [{\"from\": <node>, \"to\": <node>, "
    "\"fallback\": true}]}. Edges must point from producers to consumers; endpoints "
    "and fallback URLs are filled in from the registry.\n\n"
    "Available services:\n"
)


def service_line(s, compact: bool = False) -> str:
    ins = json.dumps(s.get("input_schema") or {}, separators=(",", ":"), sort_keys=True)
    outs = json.dumps(s.get("output_schema") or {}, separators=(",", ":"), sort_keys=True)
    if compact:
        return f"- {s['name']} (inputs: {ins}, outputs: {outs})\n"
    return f"- {s['name']} (endpoint: {s['endpoint']}, inputs: {ins}, outputs: {outs})\n"


def build_prompt_parts(services: Sequence, intent: str, compact: bool = False) -> Tuple[str, str]:
    """``compact``: the prompt of the grammar's compact model view (no URLs)."""
    prefix = (HEADER_COMPACT if compact else HEADER) + \
        "".join(service_line(s, compact) for s in services)
    suffix = f"\nUser intent: “{intent}”\n\nJSON DAG:"
    return prefix, suffix


class PromptCache:
    """Registry prefix text cached per (registry version, candidate names): the
    reference rebuilds it from every record on every call (control_plane.py:60-66)."""

    def __init__(self, maxsize: int = 256):
        self._c = {}
        self.maxsize = maxsize

    def parts(self, services: Sequence, intent: str, version=None) -> Tuple[str, str]:
        key = (version, tuple(s["name"] for s in services)) if version is not None else None
        prefix = self._c.get(key) if key is not None else None
        if prefix is None:
            prefix = HEADER + "".join(service_line(s) for s in services)
            if key is not None:
                if len(self._c) >= self.maxsize:
                    self._c.clear()
                self._c[key] = prefix
        return prefix, f"\nUser intent: “{intent}”\n\nJSON DAG:"


def build_prompt(services: Sequence, intent: str) -> str:
    p, s = build_prompt_parts(services, intent)
    return p + s


SYNTHETIC_INTENTS: List[str] = [
    "charge the customer for order {i} and email the receipt",
    "validate the shipping address for user {i} then quote shipping",
    "score order {i} for fraud and reserve inventory if clean",
    "look up the profile of user {i} and recommend products",
    "convert the invoice {i} total to EUR and file it in the ledger",
    "verify kyc for user {i}, then create an account and notify them by sms",
    "search the catalog for item {i}, price it with tax and add it to the cart",
    "aggregate analytics for region {i} and render a weekly report",
]


def synthetic_intent(i: int) -> str:
    return SYNTHETIC_INTENTS[i % len(SYNTHETIC_INTENTS)].format(i=1000 + i)
