from .records import ServiceRecord, make_service, synthetic_registry
from .registry import BaseRegistry, MemoryRegistry, RedisRegistry, make_registry
from .resp import RespClient, RespServer

__all__ = ["ServiceRecord", "make_service", "synthetic_registry", "BaseRegistry",
           "MemoryRegistry", "RedisRegistry", "make_registry", "RespClient", "RespServer"]
