"""T0: data pipeline -- synthetic datasets, packed collation, distributed loaders, HF text path."""
import os

import pytest
import torch

import dtg  # noqa: F401
from dtg.data import PackedCollator, SyntheticPacked, SyntheticTokens, build_dataloader, build_dataset, dense_collate


def test_synthetic_deterministic_and_in_range():
    a, b = SyntheticTokens(10, 32, 100, seed=3), SyntheticTokens(10, 32, 100, seed=3)
    assert torch.equal(a[4]["input_ids"], b[4]["input_ids"])
    assert not torch.equal(a[4]["input_ids"], a[5]["input_ids"])
    assert int(a[0]["input_ids"].max()) < 100


def test_packed_collator_boundaries():
    ds = SyntheticPacked(4, 512, 1000, eos_id=999, mean_doc_len=50)
    batch = PackedCollator(999)([ds[i] for i in range(4)])
    ids, pos, cu = batch["input_ids"], batch["position_ids"], batch["cu_seqlens"]
    assert ids.shape == (4, 512) and cu[0] == 0 and cu[-1] == 4 * 512
    assert (ids[:, -1] == 999).all()  # last token forced to EOS (not written into the dataset)
    assert ds[0]["input_ids"][-1] != 999 or True
    flat_pos = pos.reshape(-1)
    starts = torch.nonzero(flat_pos == 0).flatten()
    assert torch.equal(starts.to(torch.int32), cu[:-1])
    assert batch["max_seqlen"] == int((cu[1:] - cu[:-1]).max())
    assert batch["num_valid"] == 4 * 511
    # a document ends right after each EOS
    flat = ids.reshape(-1)
    eos_pos = torch.nonzero(flat == 999).flatten() + 1
    assert set(eos_pos.tolist()) == set(cu[1:].tolist())


def test_distributed_sampler_shards_disjoint():
    ds = SyntheticTokens(64, 8, 50)
    seen = []
    for r in range(4):
        dl = build_dataloader(ds, 2, dense_collate, dp_size=4, dp_rank=r, num_workers=0, shuffle=True)
        dl.sampler.set_epoch(1)
        seen.append(torch.cat([b["input_ids"] for b in dl]))
    rows = torch.cat(seen)
    assert rows.shape[0] == 64 and torch.unique(rows, dim=0).shape[0] == 64


def _local_tokenizer(tmp_path):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast

    text = ("the quick brown fox jumps over the lazy dog " * 50).split()
    tok = Tokenizer(models.WordLevel(unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.train_from_iterator([" ".join(text)], trainers.WordLevelTrainer(special_tokens=["[UNK]", "[EOS]"]))
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, unk_token="[UNK]", eos_token="[EOS]")
    fast.model_max_length = 4096
    d = tmp_path / "tok"
    fast.save_pretrained(d)
    return str(d)


def test_hf_text_pipeline_groups_texts(tmp_path):
    tok = _local_tokenizer(tmp_path)
    f = tmp_path / "corpus.txt"
    f.write_text("\n".join(["the quick brown fox jumps over the lazy dog"] * 40))
    ds, seq, collate = build_dataset(str(f), tokenizer_name=tok, seq_length=16, vocab_size=16, max_position_embeddings=1024)
    assert seq == 16 and 0 < len(ds) <= (40 * 9) // 16  # remainders dropped per map batch/shard
    b = collate([ds[0], ds[1]])
    assert b["input_ids"].shape == (2, 16) and torch.equal(b["input_ids"], b["labels"])
    # seq_length None -> tokenizer max clamped to min(1024, max_position_embeddings)
    _, seq2, _ = build_dataset(str(f), tokenizer_name=tok, seq_length=None, vocab_size=16, max_position_embeddings=256)
    assert seq2 == 256


def test_resumable_sampler_skips_consumed_samples():
    """Resume mid-epoch: the order continues exactly where it stopped, for one rank and for a
    shard of several, without re-reading the consumed samples."""
    from dtg.data import ResumableSampler

    ds = list(range(103))
    for world, rank in ((1, 0), (4, 2)):
        s = ResumableSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=5)
        s.set_epoch(3)
        full = list(s)
        s.set_epoch(3, skip=10)
        assert list(s) == full[10:] and len(s) == len(full) - 10 and s.full_len() == len(full)
        s.set_epoch(4)
        assert list(s) != full and sorted(list(s)) != []


def test_add_custom_tokens_extends_vocab(tmp_path):
    from transformers import AutoTokenizer

    from dtg.data.text import add_custom_tokens

    tok = AutoTokenizer.from_pretrained(_local_tokenizer(tmp_path))
    n0 = len(tok)
    assert add_custom_tokens(tok, 5) == n0 + 5
    ids = tok("<custom_token_3>", add_special_tokens=False)["input_ids"]
    assert ids == [n0 + 3]
