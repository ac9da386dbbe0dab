"""Service record schema (wire format T1).

Reference: the JSON value stored at ``mcp:service:<name>`` documented at
control_plane.py:31 and README.md:86-95:
``{name, endpoint, input_schema, output_schema, cost_profile, fallback}``.
Unknown keys are preserved (``extra``) so records round-trip byte-for-byte
through the registry.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional


class ServiceRecord(dict):
    """A ``dict`` subclass so records serialise exactly as stored."""

    REQUIRED = ("name", "endpoint")

    @classmethod
    def parse(cls, raw) -> "ServiceRecord":
        if isinstance(raw, (bytes, bytearray)):
            raw = raw.decode("utf-8")
        obj = json.loads(raw) if isinstance(raw, str) else dict(raw)
        if not isinstance(obj, dict):
            raise ValueError("service record must be a JSON object")
        for k in cls.REQUIRED:
            if k not in obj:
                raise ValueError(f"service record missing '{k}'")
        return cls(obj)

    @property
    def name(self) -> str:
        return self["name"]

    @property
    def endpoint(self) -> str:
        return self["endpoint"]

    @property
    def input_schema(self) -> Dict[str, Any]:
        return self.get("input_schema") or {}

    @property
    def output_schema(self) -> Dict[str, Any]:
        return self.get("output_schema") or {}

    @property
    def fallback(self) -> Optional[str]:
        return self.get("fallback")

    def input_keys(self) -> List[str]:
        """Input field names: JSON-Schema ``properties`` or a flat {key: type} map."""
        sch = self.input_schema
        if isinstance(sch, dict) and isinstance(sch.get("properties"), dict):
            return list(sch["properties"].keys())
        if isinstance(sch, dict):
            return [k for k in sch.keys() if k not in ("type", "required", "$schema", "title")]
        return []

    def schema_text(self) -> str:
        """Text used to embed the service for retrieval (the pgvector role)."""
        return (f"{self.name} inputs {json.dumps(self.input_schema, sort_keys=True)} "
                f"outputs {json.dumps(self.output_schema, sort_keys=True)}")

    def dumps(self) -> str:
        return json.dumps(self, separators=(",", ":"))


def make_service(name: str, inputs=None, outputs=None, cost: float = 0.001,
                 fallback: Optional[str] = None, endpoint: Optional[str] = None) -> ServiceRecord:
    """Convenience constructor used by tests, benchmarks and the demo registry."""
    inputs = inputs or {}
    outputs = outputs or {}
    return ServiceRecord({
        "name": name,
        "endpoint": endpoint or f"http://{name}-service/api",
        "input_schema": {"type": "object", "properties": {k: {"type": v} for k, v in inputs.items()}},
        "output_schema": {"type": "object", "properties": {k: {"type": v} for k, v in outputs.items()}},
        "cost_profile": cost,
        "fallback": fallback if fallback is not None else f"http://{name}-fallback/api",
    })


_DOMAINS = ["user", "order", "payment", "inventory", "shipping", "email", "sms", "fraud",
            "catalog", "pricing", "tax", "invoice", "auth", "profile", "search", "recommend",
            "review", "loyalty", "coupon", "cart", "geo", "weather", "currency", "translate",
            "ocr", "kyc", "ledger", "audit", "notify", "report", "analytics", "billing"]
_VERBS = ["lookup", "validate", "create", "score", "fetch", "enrich", "quote", "charge",
          "reserve", "dispatch", "render", "verify", "rank", "sync", "resolve", "aggregate"]
_FIELDS = ["user_id", "order_id", "amount", "currency", "sku", "address", "email", "phone",
           "token", "score", "items", "query", "locale", "country", "invoice_id", "status"]


def synthetic_registry(n: int, seed: int = 0) -> List[ServiceRecord]:
    """Deterministic synthetic registry of ``n`` services (benchmarks, tests)."""
    import random
    rng = random.Random(seed)
    out, seen = [], set()
    i = 0
    while len(out) < n:
        d = _DOMAINS[i % len(_DOMAINS)]
        v = _VERBS[(i // len(_DOMAINS)) % len(_VERBS)]
        name = f"{d}-{v}" if i < len(_DOMAINS) * len(_VERBS) else f"{d}-{v}-{i}"
        i += 1
        if name in seen:
            continue
        seen.add(name)
        ins = {f: rng.choice(["string", "number"]) for f in rng.sample(_FIELDS, rng.randint(1, 3))}
        outs = {f: rng.choice(["string", "number", "object"]) for f in rng.sample(_FIELDS, rng.randint(1, 2))}
        out.append(make_service(name, ins, outs, cost=round(rng.uniform(0.0005, 0.02), 4)))
    return out
