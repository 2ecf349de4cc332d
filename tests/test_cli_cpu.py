"""T0: chapter command lines keep the reference's flags and defaults."""
import pytest

import dtg  # noqa: F401
from dtg.train.cli import get_parser

BASE = ["-e", "x", "-d", "synthetic", "-m", "gpt2"]


@pytest.mark.parametrize("chapter", ["01", "02", "04", "05", "06", "07"])
def test_common_defaults(chapter):
    a = get_parser(chapter).parse_args(BASE)
    assert (a.save_dir, a.seed, a.num_epochs, a.lr, a.batch_size, a.log_freq, a.ckpt_freq, a.seq_length) == \
        ("../outputs", 0, 100, 3e-5, 1, 100, 500, 1024)
    long = get_parser(chapter).parse_args(["--experiment-name", "x", "--dataset-name", "d", "--model-name", "m",
                                           "--batch-size", "4", "--seq-length", "2048"])
    assert long.batch_size == 4 and long.seq_length == 2048


def test_required_flags():
    for ch in ("01", "04", "07"):
        with pytest.raises(SystemExit):
            get_parser(ch).parse_args(["-e", "x"])


def test_chapter_specific_flags():
    a = get_parser("04").parse_args(BASE)
    assert a.numel_to_wrap == 100_000_000 and a.cpu_offload == "off"
    assert get_parser("05").parse_args(BASE).cpu_offload == "on"
    assert get_parser("05").parse_args(BASE).activation_checkpointing == "on"
    assert get_parser("07").parse_args(BASE).tp == 8
    assert get_parser("07").parse_args(BASE + ["--tp", "1"]).tp == 1  # allowed here
    assert get_parser("06").parse_args(BASE).seq_length == 1024  # not None
    assert get_parser("02").parse_args(BASE).dp_mode == "zero"


def test_rime_and_deepspeed():
    r = get_parser("rime").parse_args(["-e", "x"])
    assert (r.num_epochs, r.log_freq, r.seq_length, r.model_name) == (1, 50, 8192, "llama-3.2-3b-rime")
    d = get_parser("deepspeed").parse_args(BASE + ["--deepspeed", "--deepspeed_config", "cfg.json", "--local_rank", "3"])
    assert d.deepspeed and d.deepspeed_config == "cfg.json" and d.local_rank == 3


def test_deepspeed_config_mapping(tmp_path):
    import json

    from dtg.train.trainer import _deepspeed_overrides

    cfg = tmp_path / "ds.json"
    cfg.write_text(json.dumps({"train_micro_batch_size_per_gpu": 4, "optimizer": {"type": "AdamW", "params": {"lr": 1e-4}},
                               "scheduler": {"type": "WarmupCosineLR", "params": {"total_num_steps": 100}},
                               "zero_optimization": {"stage": 2}}))
    a = get_parser("deepspeed").parse_args(BASE + ["--deepspeed_config", str(cfg)])
    a = _deepspeed_overrides(a)
    assert a.batch_size == 4 and a.lr == 1e-4 and a.zero_stage == 2 and a.cpu_offload == "off"
    cfg.write_text(json.dumps({"zero_optimization": {"stage": 3, "offload_optimizer": {"device": "cpu"}}}))
    a = _deepspeed_overrides(get_parser("deepspeed").parse_args(BASE + ["--deepspeed_config", str(cfg)]))
    assert a.zero_stage == 3 and a.cpu_offload == "on"
