"""Loader for the in-tree native extension `_C.so` (built by `csrc/build.py`).

On a machine with a GPU the extension is REQUIRED: every GPU op dispatches to a gfx950 HIP
kernel, and a missing or stale build raises instead of silently falling back to eager
PyTorch.  On a CPU-only machine the CPU reference implementations are used.
"""
import os

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DTG_NATIVE_SO: load an A/B build variant instead (csrc/build.py --out ...)
SO_PATH = os.environ.get("DTG_NATIVE_SO") or os.path.join(_PKG, "_C.so")
LOADED = False
LOAD_ERROR = None


def load(required: bool | None = None) -> bool:
    global LOADED, LOAD_ERROR
    if LOADED:
        return True
    if required is None:
        required = torch.cuda.is_available() and os.environ.get("DTG_ALLOW_NO_NATIVE", "0") != "1"
    if os.path.exists(SO_PATH):
        try:
            torch.ops.load_library(SO_PATH)
            LOADED = True
            return True
        except OSError as e:  # pragma: no cover - only on broken builds
            LOAD_ERROR = e
    else:
        LOAD_ERROR = FileNotFoundError(SO_PATH)
    if required:
        raise RuntimeError(
            f"dtg native extension could not be loaded ({LOAD_ERROR}); build it with `python csrc/build.py`"
        )
    return False


def require():
    if not LOADED:
        load(required=True)
