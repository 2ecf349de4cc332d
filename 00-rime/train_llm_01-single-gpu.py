#!/usr/bin/env python3
"""Chapter rime trainer (MI355X), under the reference's file name (00-rime/train_llm_01-single-gpu.py).

    python train_llm.py --help
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import dtg  # noqa: E402,F401
from dtg.train.trainer import main  # noqa: E402

if __name__ == "__main__":
    main("rime")
