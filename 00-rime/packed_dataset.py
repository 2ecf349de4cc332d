#!/usr/bin/env python3
"""Packed-sequence collation + loader benchmark, under the reference's file name
(00-rime/packed_dataset.py).  The collator is `dtg.data.PackedCollator` (O(T) position ids and
cu_seqlens instead of the reference's discarded O(T^2) mask); the benchmark is
tools/bench_dataloader.py:

    python packed_dataset.py
    torchrun --standalone --nproc-per-node=8 packed_dataset.py
"""
import os
import runpy
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import dtg  # noqa: E402,F401
from dtg.data import PackedCollator  # noqa: E402,F401  (re-exported for `from packed_dataset import ...`)

if __name__ == "__main__":
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools", "bench_dataloader.py"),
                   run_name="__main__")
