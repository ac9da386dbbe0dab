"""Import alias for the framework package.

The package lives in the directory
``autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd/``,
whose name is not a valid Python identifier.  Importing ``mcp_amd`` loads that
directory as a regular package (all intra-package imports are relative), so
``import mcp_amd.engine.engine`` and friends work from the repo root.
"""
import importlib.util as _ilu
import pathlib as _pl
import sys as _sys

PACKAGE_DIR = _pl.Path(__file__).resolve().parent / (
    "autonomous-microservice-composition-via-llm-agents-in-an-mcp-control-plane_amd")

_spec = _ilu.spec_from_file_location(
    __name__, PACKAGE_DIR / "__init__.py", submodule_search_locations=[str(PACKAGE_DIR)])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
