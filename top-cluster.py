#!/usr/bin/env python3
"""Cluster GPU monitor (reference: top-cluster.py). Implementation: tools/top_cluster.py (amd-smi over ssh)."""
import os
import runpy
import sys

if __name__ == "__main__":
    sys.argv[0] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "top_cluster.py")
    runpy.run_path(sys.argv[0], run_name="__main__")
