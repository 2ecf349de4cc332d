"""Reference doc/code drift that must not be replicated: every relative
markdown link in the guide resolves, no chapter README points at the reference's stale
directory names, and the SLURM script uses real `#SBATCH` directives and an existing entry point."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# inputs / blueprints written about the reference, not guide pages
NOT_GUIDE = {"SURVEY.md", "PAPERS.md", "SNIPPETS.md", "BASELINE.md", "VERDICT.md", "ADVICE.md"}
STALE = ["03-multi-node", "06-2d-parallel", "96-elastic-training", "04-sharding-fsdp", "05-sharding-deepspeed"]


def _guide_pages():
    for dp, dns, fns in os.walk(ROOT):
        dns[:] = [d for d in dns if not d.startswith(".") and d not in ("gpurun_out", "build", "__pycache__")]
        for f in fns:
            if f.endswith(".md") and f not in NOT_GUIDE and f != "PARITY.md":
                yield os.path.join(dp, f)


def test_guide_has_chapter_readmes():
    pages = {os.path.relpath(p, ROOT) for p in _guide_pages()}
    for ch in ("00-rime", "01-single-gpu", "02-distributed-data-parallel", "03-job-launchers",
               "04-fully-sharded-data-parallel", "05-training-llama-405b", "06-tensor-parallel", "07-2d-parallel"):
        assert f"{ch}/README.md" in pages


def test_relative_markdown_links_resolve():
    bad = []
    for p in _guide_pages():
        d = os.path.dirname(p)
        for m in re.finditer(r"\]\(([^)#\s]+)(#[^)]*)?\)", open(p).read()):
            t = m.group(1)
            if re.match(r"[a-z]+://|mailto:", t):
                continue
            if not os.path.exists(os.path.normpath(os.path.join(d, t))):
                bad.append((os.path.relpath(p, ROOT), t))
    assert not bad, bad


def test_no_stale_reference_paths():
    hits = [(os.path.relpath(p, ROOT), s) for p in _guide_pages() for s in STALE if s in open(p).read()]
    assert not hits, hits


def test_sbatch_directives_and_entry_point():
    text = open(os.path.join(ROOT, "03-job-launchers", "job.sbatch")).read()
    assert not re.search(r"^#\s+SBATCH", text, re.M), "'# SBATCH' (with a space) is not a slurm directive"
    assert len(re.findall(r"^#SBATCH ", text, re.M)) >= 3
    scripts = re.findall(r"\.\./([\w.-]+/train_llm\.py)", text)
    assert scripts
    for s in scripts:
        assert os.path.exists(os.path.join(ROOT, s)), s


@pytest.mark.parametrize("chapter", ["00-rime", "01-single-gpu", "02-distributed-data-parallel",
                                     "04-fully-sharded-data-parallel", "05-training-llama-405b",
                                     "06-tensor-parallel", "07-2d-parallel"])
def test_chapter_entry_points_exist(chapter):
    d = os.path.join(ROOT, chapter)
    assert any(f.startswith("train_llm") and f.endswith(".py") for f in os.listdir(d))


def test_cited_profile_files_exist():
    """Every `profiles/<file>` a guide page, PARITY.md or a profile note cites must exist: the
    numbers in the chapters are only as good as the evidence they point at."""
    pages = list(_guide_pages()) + [os.path.join(ROOT, "PARITY.md")]
    bad = []
    for p in pages:
        for m in re.finditer(r"profiles/([\w.\-/*]+[\w*])", open(p).read()):
            t = m.group(1)
            if t.endswith("NN.sh"):
                continue
            if not glob.glob(os.path.join(ROOT, "profiles", t)):
                bad.append((os.path.relpath(p, ROOT), t))
    assert not bad, bad
