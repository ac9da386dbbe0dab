"""Typed settings.

The reference reads three environment variables (control_plane.py:17-19) and
hard-codes everything else (key prefix :20, model/temperature :70-72, timeout
:109/:123, host/port :157).  We keep the env var names ``REDIS_URL`` and
``POSTGRES_DSN`` (the latter is accepted but unused: the schema-embedding store
lives in HBM, see ``retrieval``) and expose the rest as ``MCP_*`` variables.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

SERVICES_PREFIX = "mcp:service:"
TELEMETRY_PREFIX = "mcp:telemetry:"


def _env(name: str, default, cast=str):
    raw = os.getenv(name)
    if raw is None or raw == "":
        return default
    if cast is bool:
        return raw.strip().lower() in ("1", "true", "yes", "on")
    return cast(raw)


@dataclasses.dataclass
class Settings:
    # registry
    redis_url: Optional[str] = None          # None -> in-memory registry
    postgres_dsn: Optional[str] = None       # accepted for parity, unused
    services_prefix: str = SERVICES_PREFIX
    synthetic_services: int = 0              # >0 and no Redis: seed the in-memory registry (benches, demos)
    # planner
    planner_backend: str = "stub"            # stub | local | openai
    openai_base_url: str = "https://api.openai.com/v1"   # openai backend (reference parity)
    openai_api_key: Optional[str] = None     # OPENAI_API_KEY (control_plane.py:19)
    remote_model: str = "gpt-4o-mini"        # control_plane.py:70
    plan_cache: int = 0                      # >0: LRU plan cache entries (intent, registry version)
    model: str = "llama3-8b"                 # llama3-8b | llama3-70b | tiny
    tp: int = 1                              # >1: this process is TP rank 0, workers spawned (parallel.tp_serve)
    replicas: int = 1
    router: bool = False                     # DP router + replica processes even at replicas == 1
    api_workers: int = 1                     # >1: API worker processes on one SO_REUSEPORT port,
                                             # each routing to its own slice of the replicas
    replica_slice: Optional[str] = None      # "w/n": this API worker's slice (set by the supervisor)
    max_batch: int = 256
    max_step_tokens: int = 8192
    kv_blocks: int = 0                       # 0 -> size from free HBM
    temperature: float = 0.2                 # control_plane.py:72
    max_nodes: int = 6
    min_nodes: int = 1
    topk: int = 32                           # schema retrieval: services kept in prompt
    retrieval_threshold: int = 48            # prune only when registry is larger
    embed_dim: int = 1024
    seed: int = 0
    # orchestrator
    exec_timeout: float = 5.0                # control_plane.py:109,123
    retries: int = 0                         # parity default (reference has none)
    concurrent_generations: bool = False     # parity default: strictly serial
    use_registry_fallback: bool = False      # parity default: edge fallback only
    telemetry_to_registry: bool = False
    # adaptive planning from telemetry (README.md:43-44,48; planner/audit.py)
    adaptive: bool = False
    adaptive_error_rate: float = 0.2
    adaptive_min_calls: int = 5
    adaptive_retries: int = 1

    @classmethod
    def from_env(cls) -> "Settings":
        return cls(
            redis_url=_env("REDIS_URL", None),
            postgres_dsn=_env("POSTGRES_DSN", None),
            synthetic_services=_env("MCP_SYNTHETIC_SERVICES", 0, int),
            planner_backend=_env("MCP_PLANNER_BACKEND", "stub"),
            openai_base_url=_env("OPENAI_BASE_URL", "https://api.openai.com/v1"),
            openai_api_key=_env("OPENAI_API_KEY", None),
            remote_model=_env("MCP_REMOTE_MODEL", "gpt-4o-mini"),
            plan_cache=_env("MCP_PLAN_CACHE", 0, int),
            model=_env("MCP_MODEL", "llama3-8b"),
            tp=_env("MCP_TP", 1, int),
            replicas=_env("MCP_REPLICAS", 1, int),
            router=_env("MCP_ROUTER", False, bool),
            api_workers=_env("MCP_API_WORKERS", 1, int),
            replica_slice=_env("MCP_REPLICA_SLICE", None),
            max_batch=_env("MCP_MAX_BATCH", 256, int),
            max_step_tokens=_env("MCP_MAX_STEP_TOKENS", 8192, int),
            kv_blocks=_env("MCP_KV_BLOCKS", 0, int),
            temperature=_env("MCP_TEMPERATURE", 0.2, float),
            max_nodes=_env("MCP_MAX_NODES", 6, int),
            min_nodes=_env("MCP_MIN_NODES", 1, int),
            topk=_env("MCP_TOPK", 32, int),
            retrieval_threshold=_env("MCP_RETRIEVAL_THRESHOLD", 48, int),
            embed_dim=_env("MCP_EMBED_DIM", 1024, int),
            seed=_env("MCP_SEED", 0, int),
            exec_timeout=_env("MCP_EXEC_TIMEOUT", 5.0, float),
            retries=_env("MCP_RETRIES", 0, int),
            concurrent_generations=_env("MCP_CONCURRENT_GENERATIONS", False, bool),
            use_registry_fallback=_env("MCP_USE_REGISTRY_FALLBACK", False, bool),
            telemetry_to_registry=_env("MCP_TELEMETRY_TO_REGISTRY", False, bool),
            adaptive=_env("MCP_ADAPTIVE", False, bool),
            adaptive_error_rate=_env("MCP_ADAPTIVE_ERROR_RATE", 0.2, float),
            adaptive_min_calls=_env("MCP_ADAPTIVE_MIN_CALLS", 5, int),
            adaptive_retries=_env("MCP_ADAPTIVE_RETRIES", 1, int),
        )
