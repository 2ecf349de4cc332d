"""hipBLASLt GEMM solution selection via PyTorch TunableOp.

Plain library GEMMs (every Linear of the model) run through hipBLASLt.  Its default
heuristic picks a reasonable but not always the fastest kernel for the Llama shapes, so the
per-shape winners are measured once on an MI355X with TunableOp and committed as
`tunableop/tunableop_results.csv`; later runs load that table (no tuning cost), and only tune
shapes it does not contain when asked to (`tune=True`).
"""
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# DTG_TUNABLEOP_TABLE: an alternative table (A/B of pinned solutions, tools/tunableop_variants.py)
TABLE = os.environ.get("DTG_TUNABLEOP_TABLE") or os.path.join(ROOT, "tunableop", "tunableop_results_partial.csv")


def enable_tunableop(tune: bool = False, max_tuning_ms: int = 30, table: str = TABLE):
    os.makedirs(os.path.dirname(table), exist_ok=True)
    t = torch.cuda.tunable
    record = os.environ.get("DTG_TUNABLEOP_RECORD")
    if record:
        # list the GEMM shapes the table lacks, for offline tuning with tools/tune_gemms.py
        os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = record
        t.record_untuned_enable(True)
    t.enable(True)
    if not tune:
        # Read-only use: point TunableOp's own results file at a per-process scratch copy so
        # that no rank can rewrite the committed table at exit (8 ranks, one file).
        import shutil
        import tempfile

        scratch = os.path.join(tempfile.gettempdir(), f"dtg_tunableop_{os.getpid()}.csv")
        if os.path.exists(table):
            shutil.copyfile(table, scratch)
        table = scratch
    t.set_filename(table, insert_device_ordinal=False)
    t.tuning_enable(tune)
    if tune:
        t.set_max_tuning_duration(max_tuning_ms)
        t.set_max_tuning_iterations(50)
    if os.path.exists(table):
        t.read_file(table)


def save_tunableop(table: str = TABLE):
    """Write the tuned results now if this torch exposes `write_file`; otherwise TunableOp
    writes them to its results file (set by enable_tunableop / set_filename) at process exit."""
    t = torch.cuda.tunable
    if hasattr(t, "write_file"):
        t.write_file(table)
    elif os.path.abspath(t.get_filename()) != os.path.abspath(table):
        import warnings

        warnings.warn(f"tunableop: results go to {t.get_filename()} at exit, not {table}")
