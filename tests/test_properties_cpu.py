"""Property-based tests (hypothesis) of the host-side logic every run depends on -- SURVEY §4.2
tier T0: packed-sequence collation against a naive token walk, flat-buffer bucketing and shard
ranges, DCP name/row mapping of the fused projections, the activation-checkpointing budget,
the skip-ahead sampler, the LR schedule and LR scaling rules.

References: /root/reference/00-rime/packed_dataset.py:14-49 (collate), 02-distributed-data-
parallel/train_llm.py:96-103 (sampler), 04-fully-sharded-data-parallel/train_llm.py:249-263 (DCP
keys), 01-single-gpu/train_llm.py:111-113 (cosine schedule)."""
import argparse
import math
import os

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

# DTG_HYP_EXAMPLES raises the example count for a longer hunt (default: a few seconds in total)
SETTINGS = dict(max_examples=int(os.environ.get("DTG_HYP_EXAMPLES", "60")), deadline=None, database=None,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
EOS = 0


# ------------------------------------------------------------------------------ packing
def _naive_positions(row):
    """Walk the tokens: positions restart after every EOS; the last token ends a document."""
    pos, lens, p = [], [], 0
    for i, tok in enumerate(row):
        pos.append(p)
        p += 1
        if tok == EOS or i == len(row) - 1:
            lens.append(p)
            p = 0
    return pos, lens


@settings(**SETTINGS)
@given(st.integers(1, 4).flatmap(lambda b: st.integers(1, 48).flatmap(
    lambda t: st.lists(st.lists(st.sampled_from([EOS, 1, 2, 3, 4, 5]), min_size=t, max_size=t),
                       min_size=b, max_size=b))))
def test_packed_collate_matches_naive_walk(rows):
    from dtg.data.packed import PackedCollator

    samples = [{"input_ids": torch.tensor(r)} for r in rows]
    before = [s["input_ids"].clone() for s in samples]
    out = PackedCollator(EOS)(samples)
    T = len(rows[0])
    forced = [r[:-1] + [EOS] for r in rows]  # the reference forces x[-1] = eos
    assert out["input_ids"].tolist() == forced and out["labels"].tolist() == forced
    assert all(torch.equal(a, s["input_ids"]) for a, s in zip(before, samples))  # no in-place EOS write
    pos, lens = zip(*(_naive_positions(r) for r in forced))
    assert out["position_ids"].tolist() == list(pos)
    flat_lens = [n for ls in lens for n in ls]
    assert out["cu_seqlens"].dtype == torch.int32
    assert out["cu_seqlens"].tolist() == [0] + list(torch.cumsum(torch.tensor(flat_lens), 0).tolist())
    assert out["cu_seqlens"][-1] == len(rows) * T and out["max_seqlen"] == max(flat_lens)
    assert out["num_valid"] == len(rows) * (T - 1)
    # the documents cu_seqlens delimits are exactly the blocks where position ids restart
    doc = torch.repeat_interleave(torch.arange(len(flat_lens)), torch.tensor(flat_lens))
    starts = (out["position_ids"].reshape(-1) == 0).cumsum(0) - 1
    assert torch.equal(doc, starts)


# ------------------------------------------------------------------------------ flat buckets
@settings(**SETTINGS)
@given(st.lists(st.lists(st.integers(1, 40), min_size=1, max_size=2), min_size=1, max_size=12),
       st.integers(1, 8), st.integers(64, 4096), st.booleans())
def test_flat_space_buckets_partition_and_shard(shapes, world, bucket_bytes, with_trailing):
    from dtg.parallel.flat import ALIGN, FlatSpace

    params = [(f"p{i}", torch.nn.Parameter(torch.zeros(*s))) for i, s in enumerate(shapes)]
    trailing = (lambda p: p.dim() == 1) if with_trailing else None
    sp = FlatSpace(params, "cpu", world=world, bucket_bytes=bucket_bytes, trailing=trailing)
    # buckets tile [0, numel) contiguously, each a whole number of world x ALIGN elements
    assert sp.buckets[0].start == 0 and sp.buckets[-1].end == sp.numel
    for a, b in zip(sp.buckets, sp.buckets[1:]):
        assert a.end == b.start
    for b in sp.buckets:
        assert b.numel > 0 and b.numel % (world * ALIGN) == 0
        ranges = [sp.shard_range(b, r) for r in range(world)]
        assert ranges[0][0] == b.start and ranges[-1][1] == b.end
        assert all(x[1] == y[0] for x, y in zip(ranges, ranges[1:]))
    # every parameter is 16-element aligned, inside its own bucket, and no two overlap
    spans = []
    for i, (o, shape) in enumerate(zip(sp.offsets, sp.shapes)):
        n = math.prod(shape)
        b = sp.param_bucket[i]
        assert o % ALIGN == 0 and b.start <= o and o + n <= b.end
        spans.append((o, o + n))
        assert sp.param_view(i).shape == torch.Size(shape)
    spans.sort()
    assert all(x[1] <= y[0] for x, y in zip(spans, spans[1:]))
    # backward order: the flat order is the reverse of registration, trailing params last
    names = [n for n, _ in params][::-1]
    if with_trailing:
        tail = [n for n, p in params[::-1] if p.dim() == 1]
        names = [n for n in names if n not in tail] + tail
        if tail and len(tail) < len(params):
            assert sp.buckets[-1].trailing and all(p.dim() == 1 for p in sp.buckets[-1].params)
    assert sp.names == names


# ------------------------------------------------------------------------------ DCP names
@settings(**SETTINGS)
@given(st.sampled_from([(4, 2, 8), (8, 8, 16), (6, 2, 4), (32, 8, 16), (4, 1, 8)]), st.data())
def test_dcp_fused_projection_chunks_tile_the_rectangle(heads, data):
    """Any row range of the fused qkv / gate_up weight (a TP shard, an FSDP piece) maps onto HF
    q/k/v (gate/up) chunks that cover exactly those rows, at the right HF offsets."""
    from dtg.models.config import LlamaConfig
    from dtg.train.dcp_ckpt import _Names

    nq, nkv, d = heads
    inter = data.draw(st.integers(1, 40))
    H = 16
    cfg = LlamaConfig(vocab_size=32, hidden_size=H, intermediate_size=inter, num_hidden_layers=1,
                      num_attention_heads=nq, num_key_value_heads=nkv, head_dim=d)
    names = _Names(cfg)
    for name, rows, parts in (
            ("layers.0.self_attn.qkv_proj.weight", (nq + 2 * nkv) * d,
             [("q_proj", 0, nq * d), ("k_proj", nq * d, nkv * d), ("v_proj", (nq + nkv) * d, nkv * d)]),
            ("layers.0.mlp.gate_up_proj.weight", 2 * inter, [("gate_proj", 0, inter), ("up_proj", inter, inter)])):
        r0 = data.draw(st.integers(0, rows - 1))
        nr = data.draw(st.integers(1, rows - r0))
        c0 = data.draw(st.integers(0, H - 1))
        nc = data.draw(st.integers(1, H - c0))
        got = names.split(name, [rows, H], [r0, nr, c0, nc, 0])
        covered = []
        for hf, hshape, offs, sizes, (lo, hi) in got:
            short, g0, n = next(p for p in parts if hf.endswith(p[0] + ".weight"))
            assert hf.startswith("model.layers.0.") and hshape == [n, H]
            assert offs == [lo - g0, c0] and sizes == [hi - lo, nc]
            assert g0 <= lo < hi <= g0 + n
            covered.append((lo, hi))
        covered.sort()
        assert covered[0][0] == r0 and covered[-1][1] == r0 + nr
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


# ------------------------------------------------------------------------------ AC budget
@settings(**SETTINGS)
@given(st.integers(1, 130), st.data(), st.integers(1, 10 ** 9), st.integers(0, 10 ** 8),
       st.integers(0, 400 * 10 ** 9), st.integers(0, 400 * 10 ** 9), st.floats(1.0, 2.0))
def test_ac_budget_keeps_the_fewest_layers_that_fit(n, data, per, inp, peak, budget, safety):
    from dtg.parallel.checkpointing import ac_layers_for_budget

    n_ckpt = data.draw(st.integers(0, n))
    keep = ac_layers_for_budget(n, n_ckpt, peak, budget, per, inp, safety)
    assert 0 <= keep <= n_ckpt
    extra = max(1, int((per - inp) * safety))
    released = n_ckpt - keep
    if peak >= budget:
        assert keep == n_ckpt  # over budget already: nothing is released
    else:
        assert peak + released * extra <= budget  # what is released fits
        assert keep == 0 or peak + (released + 1) * extra > budget  # and one more would not
    # a larger budget never checkpoints more layers
    assert ac_layers_for_budget(n, n_ckpt, peak, budget + 10 ** 9, per, inp, safety) <= keep


# ------------------------------------------------------------------------------ sampler
@settings(**SETTINGS)
@given(st.integers(1, 200), st.integers(1, 8), st.integers(0, 5), st.integers(0, 3), st.data())
def test_sampler_resume_and_rank_partition(n, world, seed, epoch, data):
    from dtg.data import ResumableSampler

    ds = list(range(n))
    full = []
    for r in range(world):
        s = ResumableSampler(ds, num_replicas=world, rank=r, seed=seed)
        s.set_epoch(epoch)
        order = list(s)
        assert len(order) == len(s) == n // world  # drop_last
        full.append(order)
        skip = data.draw(st.integers(0, len(order)))
        s.set_epoch(epoch, skip=skip)  # resume part-way: the same order, minus what was consumed
        assert list(s) == order[skip:] and len(s) == len(order) - skip
    flat = [i for o in full for i in o]
    assert len(set(flat)) == len(flat)  # ranks never share a sample


# ------------------------------------------------------------------------------ LR
@settings(**SETTINGS)
@given(st.floats(1e-6, 1e-2), st.integers(0, 50), st.integers(51, 300), st.floats(0.0, 0.5))
def test_warmup_cosine_schedule(lr, warm, total, floor):
    from dtg.train.trainer import _scheduler

    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=lr)
    args = argparse.Namespace(lr=lr, ds_scheduler={"type": "WarmupCosineLR", "params": {
        "total_num_steps": total, "warmup_num_steps": warm, "cos_min_ratio": floor}})
    sched = _scheduler(args, opt)
    lrs = []
    for _ in range(total + 5):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sched.step()
    for i in range(1, warm):  # linear warm-up
        assert lrs[i] == pytest.approx(lr * (i + 1) / warm, rel=1e-6)
    assert all(0 <= x <= lr * (1 + 1e-6) for x in lrs)
    assert all(x >= floor * lr * (1 - 1e-6) for x in lrs[warm:])  # the cosine floor after warm-up
    tail = lrs[warm:total + 1]
    assert all(a >= b - 1e-12 for a, b in zip(tail, tail[1:]))  # non-increasing after warm-up
    assert lrs[-1] == pytest.approx(floor * lr, rel=1e-6, abs=1e-12)


@settings(**SETTINGS)
@given(st.floats(1e-6, 1.0), st.integers(1, 4096), st.integers(1, 4096), st.integers(1, 64), st.integers(1, 16))
def test_lr_scaling_rules(lr, b0, b1, dp, accum):
    from dtg.utils.lr_scaling import effective_batch, scale_lr

    assert effective_batch(b1, dp, accum) == b1 * dp * accum
    assert scale_lr(lr, b0, b0) == pytest.approx(lr)
    lin, sq = scale_lr(lr, b0, b1, "linear"), scale_lr(lr, b0, b1, "sqrt")
    assert lin == pytest.approx(lr * b1 / b0) and sq == pytest.approx(lr * math.sqrt(b1 / b0))
    assert (lin >= sq) == (b1 >= b0) or lin == pytest.approx(sq)
    with pytest.raises(ValueError):
        scale_lr(lr, b0, b1, "cubic")


# ------------------------------------------------------------------------------ TP geometry
def _tp_local(G, kind, r, n, nq, nkv, d):
    """The TP plan's shard of global tensor G (2-D) for rank r of n, written independently of
    train/checkpoint.py: q/k/v and gate/up row blocks per rank, o/down column blocks, embedding /
    head row blocks, everything else replicated."""
    if n == 1 or kind == "rep":
        return G
    if kind == "qkv":
        q, k, v = G[:nq * d], G[nq * d:(nq + nkv) * d], G[(nq + nkv) * d:]
        bq, bk = nq // n * d, nkv // n * d
        return torch.cat([q[r * bq:(r + 1) * bq], k[r * bk:(r + 1) * bk], v[r * bk:(r + 1) * bk]])
    if kind == "gate_up":
        i = G.shape[0] // 2
        b = i // n
        return torch.cat([G[r * b:(r + 1) * b], G[i + r * b:i + (r + 1) * b]])
    if kind == "col":
        b = G.shape[1] // n
        return G[:, r * b:(r + 1) * b]
    b = G.shape[0] // n  # row
    return G[r * b:(r + 1) * b]


@settings(**SETTINGS)
@given(st.sampled_from([1, 2, 4, 8]), st.sampled_from(["layers.0.self_attn.qkv_proj.weight", "layers.0.mlp.gate_up_proj.weight",
                                                       "layers.0.self_attn.o_proj.weight", "embed_tokens.weight",
                                                       "layers.0.input_layernorm.weight", "layers.0.self_attn.qkv_proj.bias"]),
       st.data())
def test_checkpoint_rectangles_tile_the_global_tensor(n, name, data):
    """Every rank's TP-local flat range, cut into arbitrary data-parallel pieces, maps to global
    rectangles (train/checkpoint.py _TPGeom.rects) that hold exactly the right elements and,
    over all ranks and pieces, cover the global tensor once -- what lets a checkpoint load on
    any (dp, tp) layout."""
    from dtg.models.config import LlamaConfig
    from dtg.train.checkpoint import _TPGeom, param_kind

    nkv = n * data.draw(st.integers(1, 2))
    nq = nkv * data.draw(st.integers(1, 3))
    d, H = 4, 8 * n
    inter = n * data.draw(st.integers(1, 3))
    cfg = LlamaConfig(vocab_size=16 * n, hidden_size=H, intermediate_size=inter, num_hidden_layers=1,
                      num_attention_heads=nq, num_key_value_heads=nkv, head_dim=d)
    kind = param_kind(name) if n > 1 else "rep"
    gshape = {"qkv": [(nq + 2 * nkv) * d, 1 if name.endswith("bias") else H], "gate_up": [2 * inter, H],
              "col": [H, nq * d], "row": [cfg.vocab_size, H], "rep": [1, H]}[param_kind(name)]
    G = torch.arange(math.prod(gshape), dtype=torch.float64).view(gshape)
    seen = torch.zeros(gshape, dtype=torch.int64)
    for r in range(n):
        geo = object.__new__(_TPGeom)
        geo.rank, geo.size, geo.cfg = r, n, cfg
        L = _tp_local(G, kind, r, n, nq, nkv, d).contiguous()
        local_shape = [H] if name.endswith("layernorm.weight") else list(L.shape)
        flat = L.reshape(-1)
        cuts = sorted(set(data.draw(st.lists(st.integers(1, flat.numel() - 1), max_size=4)))) if flat.numel() > 1 else []
        for start, end in zip([0] + cuts, cuts + [flat.numel()]):
            for r0, nr, c0, nc, off in geo.rects(name, local_shape, start, end - start):
                got = flat[start + off:start + off + nr * nc].view(nr, nc)
                assert torch.equal(got, G[r0:r0 + nr, c0:c0 + nc]), (r, start, (r0, nr, c0, nc, off))
                seen[r0:r0 + nr, c0:c0 + nc] += 1
    assert bool((seen == (n if kind == "rep" else 1)).all())


# ------------------------------------------------------------------------------ HF weights x TP
class _FakeHF:
    """models/loading.py's _LazyHF interface over an in-memory HF state dict."""

    def __init__(self, sd):
        self.sd = sd

    def shape(self, k):
        return list(self.sd[k].shape)

    def get(self, k):
        return self.sd[k]

    def rows(self, k, r0, r1, c0=None, c1=None):
        t = self.sd[k]
        return t[r0:r1] if (t.dim() == 1 or c0 is None) else t[r0:r1, c0:c1]


@settings(**SETTINGS)
@given(st.sampled_from([1, 2, 4]), st.booleans(), st.booleans(), st.data())
def test_hf_conversion_and_tp_loading_agree(tp, tie, bias, data):
    """HF -> fused layout -> HF is exact; the TP sharder, an independent shard rule and the
    per-rank safetensors row reader (--init-from) give the same rank-local rows for any row range."""
    from dtg.models.config import LlamaConfig
    from dtg.models.hf_compat import llama_from_hf, llama_to_hf
    from dtg.models.loading import _read_rows
    from dtg.parallel.tensor_parallel import shard_full_state_dict
    from dtg.train.checkpoint import param_kind

    nkv = tp * data.draw(st.integers(1, 2))
    nq = nkv * data.draw(st.integers(1, 2))
    d, H, inter, V = 4, 8 * tp, 4 * tp * data.draw(st.integers(1, 3)), 8 * tp
    cfg = LlamaConfig(vocab_size=V, hidden_size=H, intermediate_size=inter, num_hidden_layers=1,
                      num_attention_heads=nq, num_key_value_heads=nkv, head_dim=d, tie_word_embeddings=tie)
    g = torch.Generator().manual_seed(data.draw(st.integers(0, 10 ** 6)))
    p = "model.layers.0."
    shapes = {p + "self_attn.q_proj.weight": (nq * d, H), p + "self_attn.k_proj.weight": (nkv * d, H),
              p + "self_attn.v_proj.weight": (nkv * d, H), p + "self_attn.o_proj.weight": (H, nq * d),
              p + "mlp.gate_proj.weight": (inter, H), p + "mlp.up_proj.weight": (inter, H),
              p + "mlp.down_proj.weight": (H, inter), p + "input_layernorm.weight": (H,),
              p + "post_attention_layernorm.weight": (H,), "model.embed_tokens.weight": (V, H),
              "model.norm.weight": (H,)}
    if bias:
        shapes.update({p + "self_attn.q_proj.bias": (nq * d,), p + "self_attn.k_proj.bias": (nkv * d,),
                       p + "self_attn.v_proj.bias": (nkv * d,)})
    if not tie:
        shapes["lm_head.weight"] = (V, H)
    hf = {k: torch.randn(*s, generator=g) for k, s in shapes.items()}
    ours = llama_from_hf(hf, cfg)
    back = llama_to_hf(ours, cfg)
    assert set(back) == set(hf) | ({"lm_head.weight"} if tie else set())
    assert all(torch.equal(back[k], v) for k, v in hf.items())
    fake = _FakeHF(hf)
    for r in range(tp):
        local = shard_full_state_dict(ours, cfg, r, tp)
        for name, full in ours.items():
            kind = param_kind(name) if tp > 1 else "rep"
            G = full if full.dim() == 2 else full[None]
            mine = _tp_local(G, kind, r, tp, nq, nkv, d)
            loc = local[name] if local[name].dim() == 2 else local[name][None]
            assert torch.equal(loc, mine), (name, r)
            if name.endswith("layernorm.weight") or name == "norm.weight":
                assert torch.equal(_read_rows(fake, name, 0, H, cfg, r, tp), full)
                continue
            r0 = data.draw(st.integers(0, loc.shape[0] - 1))
            r1 = data.draw(st.integers(r0 + 1, loc.shape[0]))
            got = _read_rows(fake, name, r0, r1, cfg, r, tp)
            assert torch.equal(got.reshape(r1 - r0, -1), loc[r0:r1]), (name, r, r0, r1)
