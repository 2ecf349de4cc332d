"""GPU twin of tests/test_convergence_cpu.py: chapter 01 on `synthetic:pattern` through the HIP
kernels (flash attention at head_dim 128, fused norms / SwiGLU / CE / AdamW, hipBLASLt TN GEMMs),
eager and with the whole step captured in a HIP graph: the loss falls from ln V far down.  (The
distributed chapters' convergence runs on CPU ranks, tests/test_convergence_cpu.py; as four ranks
sharing this GPU over gloo, chapter 07 learned the same way but took 2 minutes of the GPU tier.)"""
import math

import pytest

from test_convergence_cpu import run_pattern

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph", ["off", "on"])
def test_pattern_data_is_learned_on_gpu(cuda, tmp_path, graph):
    losses = run_pattern(tmp_path, ("-m", "llama-tiny-d128", "--lr", "1e-3", "--hip-graph", graph), steps=200, timeout=300)
    assert math.log(1000) * 0.6 < losses[0]  # starts near ln V (V = 1000)
    assert losses[-1] < 1.0 and losses[-1] < losses[0] / 4, losses

