"""GPU twin of tests/test_convergence_cpu.py: chapter 01 on `synthetic:pattern` through the HIP
kernels (flash attention at head_dim 128, fused norms / SwiGLU / CE / AdamW, hipBLASLt TN GEMMs),
eager and with the whole step captured in a HIP graph, and chapter 07's FSDP x TP as four ranks
sharing the GPU (DTG_SHARED_DEVICE=1: real per-rank kernels, gloo collectives): the loss falls
from ln V far down."""
import math

import pytest

from test_convergence_cpu import run_pattern

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph", ["off", "on"])
def test_pattern_data_is_learned_on_gpu(cuda, tmp_path, graph):
    losses = run_pattern(tmp_path, ("-m", "llama-tiny-d128", "--lr", "1e-3", "--hip-graph", graph), steps=200, timeout=300)
    assert math.log(1000) * 0.6 < losses[0]  # starts near ln V (V = 1000)
    assert losses[-1] < 1.0 and losses[-1] < losses[0] / 4, losses


def test_pattern_data_is_learned_2d_on_gpu(cuda, tmp_path, monkeypatch):
    monkeypatch.setenv("DTG_SHARED_DEVICE", "1")
    losses = run_pattern(tmp_path, ("-m", "llama-tiny-d128", "--lr", "1e-3", "-b", "8", "--tp", "2"), steps=200,
                         timeout=300, chapter="07-2d-parallel", nproc=4)
    assert math.log(1000) * 0.6 < losses[0]
    assert losses[-1] < 1.0 and losses[-1] < losses[0] / 4, losses
