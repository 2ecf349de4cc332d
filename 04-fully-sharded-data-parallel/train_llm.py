#!/usr/bin/env python3
"""Chapter 04 trainer (MI355X). Same flags as the reference chapter; see README.md here.

    python train_llm.py --help
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import dtg  # noqa: E402,F401
from dtg.train.trainer import main  # noqa: E402

if __name__ == "__main__":
    main("04")
