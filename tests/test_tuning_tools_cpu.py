"""CPU checks of the GEMM-tuning tools' bookkeeping (no GPU): the sustained-load re-ranker's
parser of TunableOp's verbose log (tools/tunableop_sustained.py) and its table substitution."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# An excerpt of PyTorch 2.10's PYTORCH_TUNABLEOP_VERBOSE=3 output (profiles/r4/s31 format).
LOG = """finding fastest for GemmTunableOp_BFloat16_TN(tn_4096_16384_4096_ld_4096_4096_4096) out of 17823 candidates
├──tuning using warmup iters 0 [0 ms] and tuning iters 30 [8.39624 ms] instance id=0, GemmTunableOp_BFloat16_TN(tn_4096_16384_4096_ld_4096_4096_4096) Default
├──found better instance id=0. 0.26378ms. Default min 0.259122 max 0.271403 mean 0.26378 std 0.00404639
├──skip slow instance id=4366, GemmTunableOp_BFloat16_TN(tn_4096_16384_4096_ld_4096_4096_4096) Gemm_Rocblas_618386
├──tuning using warmup iters 0 [0 ms] and tuning iters 30 [7.83356 ms] instance id=13243, GemmTunableOp_BFloat16_TN(tn_4096_16384_4096_ld_4096_4096_4096) Gemm_Hipblaslt_618611
├──tuning using warmup iters 0 [0 ms] and tuning iters 30 [8.74797 ms] instance id=17822, GemmTunableOp_BFloat16_TN(tn_4096_16384_4096_ld_4096_4096_4096) Default
├──tuning using warmup iters 0 [0 ms] and tuning iters 16 [28.7188 ms] instance id=14103, GemmTunableOp_BFloat16_TN(tn_28672_16384_4096_ld_4096_4096_28672) Gemm_Hipblaslt_618464
"""


def test_parse_candidates_ranks_survivors():
    import tunableop_sustained as ts

    c = ts.parse_candidates(LOG)
    small = c["tn_4096_16384_4096_ld_4096_4096_4096"]
    # per-iteration mean = bracket / iterations; "Default" kept at its faster instance; skipped
    # instances are not candidates
    assert [s for s, _ in small] == ["Gemm_Hipblaslt_618611", "Default"]
    assert abs(small[0][1] - 7.83356 / 30) < 1e-5 and abs(small[1][1] - 8.39624 / 30) < 1e-5
    assert c["tn_28672_16384_4096_ld_4096_4096_28672"] == [("Gemm_Hipblaslt_618464", round(28.7188 / 16, 5))]


def test_step_shapes_keys_match_the_table():
    """Every shape the tool times is a TN key of the committed table (the step's GEMMs)."""
    import tunableop_sustained as ts

    keys = {l.split(",")[1] for l in open(ts.TABLE) if l.startswith("GemmTunableOp_BFloat16_TN")}
    for name, (m, n, k) in ts.STEP_SHAPES.items():
        assert ts.key_of(m, n, k) in keys, name
