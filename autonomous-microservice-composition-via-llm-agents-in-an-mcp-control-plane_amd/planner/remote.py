"""OpenAI-compatible remote planner (the reference's backend, kept behind a
flag: ``MCP_PLANNER_BACKEND=openai``).

Reference: ``GraphPlanner.plan`` (control_plane.py:57-75) sends the whole
prompt as one system message to ``gpt-4o-mini`` at temperature 0.2 and
``json.loads`` the reply.  This backend does the same against any
OpenAI-compatible ``/chat/completions`` endpoint (``OPENAI_BASE_URL``,
``OPENAI_API_KEY``, ``MCP_REMOTE_MODEL``) with an async httpx client, so the
event loop never blocks and the pre-1.0 SDK is not needed (D2).
Error semantics are the reference's: a reply that is not a JSON object raises
(HTTP 500 at the API).  Unlike the on-node planner nothing constrains the
reply to the T2 DAG schema.
"""
from __future__ import annotations

import json
import time
from typing import Optional

import httpx

from ..utils.metrics import METRICS
from .base import Planner
from .prompt import PromptCache


class RemotePlanner(Planner):
    def __init__(self, registry, base_url: str = "https://api.openai.com/v1",
                 api_key: Optional[str] = None, model: str = "gpt-4o-mini",
                 temperature: float = 0.2, timeout: float = 60.0,
                 transport: Optional[httpx.AsyncBaseTransport] = None):
        self.registry = registry
        self.model = model
        self.temperature = temperature
        headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}
        self._client = httpx.AsyncClient(base_url=base_url.rstrip("/"), headers=headers,
                                         timeout=timeout, transport=transport)
        self._prompts = PromptCache()
        self.last_prompt: Optional[str] = None

    async def plan(self, intent: str) -> dict:
        t0 = time.perf_counter()
        services = self.registry.list_services()
        prefix, suffix = self._prompts.parts(services, intent, getattr(self.registry, "version", None))
        prompt = self.last_prompt = prefix + suffix
        body = {"model": self.model, "temperature": self.temperature,
                "messages": [{"role": "system", "content": prompt}]}    # control_plane.py:69-73
        r = await self._client.post("/chat/completions", json=body)
        r.raise_for_status()
        text = r.json()["choices"][0]["message"]["content"]
        dag = json.loads(text)                                          # control_plane.py:74
        if not isinstance(dag, dict):
            raise ValueError(f"planner reply is not a JSON object: {type(dag).__name__}")
        METRICS.plan_done(time.perf_counter() - t0)
        return dag

    async def aclose(self):
        await self._client.aclose()
