#!/usr/bin/env python3
"""Prepare local weights for the 405B chapter (reference: download.py).

The GPU boxes have no network, so this script does not download: it validates a local HF
checkout (config.json + model-*.safetensors), reports its size/parameter count against the
bundled config, and prints the `--init-from` flag to pass.  Each rank later memory-maps only the
slices it owns (dtg.models.loading), so node-local NVMe is recommended (the reference measured
50 min from a shared drive vs 3 min node-local).
"""
import argparse
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import dtg  # noqa: E402,F401
from dtg.models import resolve_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="local directory with config.json and *.safetensors")
    ap.add_argument("--model-name", default="meta-llama/Llama-3.1-405B")
    a = ap.parse_args()
    cfg = resolve_config(a.model_name)
    files = sorted(glob.glob(os.path.join(a.path, "*.safetensors")))
    if not files:
        print(f"no *.safetensors under {a.path}; bundled config only ({cfg.num_params() / 1e9:.1f}B params)")
        return 1
    size = sum(os.path.getsize(f) for f in files)
    if os.path.exists(os.path.join(a.path, "config.json")):
        with open(os.path.join(a.path, "config.json")) as fp:
            hf = json.load(fp)
        for k in ("hidden_size", "num_hidden_layers", "num_attention_heads", "num_key_value_heads", "vocab_size"):
            if hf.get(k) != getattr(cfg, k):
                print(f"WARNING: {k} differs: checkpoint {hf.get(k)} vs bundled {getattr(cfg, k)}")
    print(f"{len(files)} files, {size / 1e9:.1f} GB; expected ~{2 * cfg.num_params() / 1e9:.1f} GB in bf16")
    print(f"pass: --init-from {os.path.abspath(a.path)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
