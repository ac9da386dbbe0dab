from .executor import Orchestrator
from .validate import DagValidationError, validate_dag, normalize_dag

__all__ = ["Orchestrator", "DagValidationError", "validate_dag", "normalize_dag"]
