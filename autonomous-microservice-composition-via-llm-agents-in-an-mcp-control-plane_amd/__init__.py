"""MI355X-native microservice-composition control plane.

Layers:

* ``api``           FastAPI surface: /plan, /execute, /plan_and_execute, /metrics
* ``registry``      service registry (in-memory + Redis/RESP backends)
* ``orchestrator``  DAG executor: generational topo order, retries, ordered fallbacks
* ``planner``       prompt builder, tokenizer, DAG grammar, planner backends
* ``engine``        paged-KV continuous-batching LLM engine (HIP kernels, hipGraph)
* ``models``        Llama-3 family (8B / 70B / tiny test configs)
* ``ops``           Python bindings of the hand-written gfx950 HIP kernels
* ``parallel``      tensor parallelism over RCCL, data-parallel replica router
* ``retrieval``     HBM-resident service-schema embedding store + top-k cosine
* ``utils``         logging, metrics, timing helpers
"""

__version__ = "0.1.0"
