"""Import shim: exposes the `lambda-labs_distributed-training-guide_amd/` package as `dtg`.

The package directory keeps the project's canonical (hyphenated) name, which is not a
valid Python identifier; this module registers it under the importable name `dtg` so
`import dtg`, `from dtg.models import llama`, multiprocessing spawn and pickling all work.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "lambda-labs_distributed-training-guide_amd")
_spec = _ilu.spec_from_file_location("dtg", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["dtg"] = _mod
_spec.loader.exec_module(_mod)
