"""Operator schemas of the `dtg` library.

Schemas are declared once here; implementations register against them:
  * CUDA (= HIP on ROCm): the gfx950 kernels in csrc/kernels/*.hip (`_C.so`)
  * CPU: fp32 PyTorch reference implementations in `dtg.ops._cpu` (tests, CPU plumbing runs)
PyTorch's dispatcher picks the implementation from the tensors' device.
"""
import torch

LIB = torch.library.Library("dtg", "DEF")

_DEFS = [
    "rmsnorm_fwd(Tensor x, Tensor w, float eps) -> (Tensor, Tensor)",
    "add_rmsnorm_fwd(Tensor x, Tensor residual, Tensor w, float eps) -> (Tensor, Tensor, Tensor)",
    "rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres) -> (Tensor, Tensor)",
    "rope_(Tensor(a!) qkv, Tensor cos, Tensor sin, Tensor pos, int nheads, int head_dim, bool inverse) -> ()",
    "swiglu_fwd(Tensor gu) -> Tensor",
    "swiglu_bwd(Tensor dh, Tensor gu) -> Tensor",
    "swiglu_bwd_t(Tensor dh, Tensor gu) -> (Tensor, Tensor, Tensor)",
    "ce_fwd_bwd_(Tensor(a!) logits, Tensor labels, int ignore_index, float grad_scale, bool compute_grad) -> Tensor",
    "ce_stats(Tensor logits, Tensor labels, int vocab_start) -> (Tensor, Tensor, Tensor)",
    "ce_grad_(Tensor(a!) logits, Tensor labels, Tensor lse, int vocab_start, int ignore_index, float grad_scale) -> ()",
    "adamw_(Tensor(a!) p, Tensor(b!)? master, Tensor g, Tensor(c!) m, Tensor(d!) v, float lr, float beta1, "
    "float beta2, float eps, float wd, int step, float grad_scale, Tensor? hyper=None) -> ()",
    # AdamW over the matrices `mats` (int64 [n, 5]: offset, rows, cols, transposed offset or -1,
    # first tile, counted in 64 x tile_cols tiles) of the flat buffers, also writing each matrix's
    # transpose into `pt`
    "adamw_t_(Tensor(a!) p, Tensor(b!)? master, Tensor g, Tensor(c!) m, Tensor(d!) v, Tensor(e!) pt, Tensor mats, "
    "int ntiles, float lr, float beta1, float beta2, float eps, float wd, int step, float grad_scale, "
    "Tensor? hyper=None, int tile_cols=64) -> ()",
    "adamw_cpu_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, float lr, float beta1, float beta2, "
    "float eps, float wd, int step, float grad_scale) -> ()",
    # window > 0 (causal only): sliding window, query i sees keys (i - window, i]
    "flash_attn_fwd(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens, int max_seqlen, float scale, bool causal, "
    "int window=0) -> (Tensor, Tensor)",
    "flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor cu_seqlens, "
    "int max_seqlen, float scale, bool causal, int window=0) -> (Tensor, Tensor, Tensor)",
    "flash_attn_bwd_qkv(Tensor dout, Tensor qkv, int nq, int nkv, int head_dim, Tensor o, Tensor lse, "
    "Tensor cu_seqlens, int max_seqlen, float scale, bool causal, int window=0) -> Tensor",
    # the same with the RoPE backward of the q / k heads fused into the dQ / dK epilogues
    "flash_attn_bwd_qkv_rope(Tensor dout, Tensor qkv, int nq, int nkv, int head_dim, Tensor o, Tensor lse, "
    "Tensor cu_seqlens, int max_seqlen, float scale, bool causal, Tensor cos, Tensor sin, Tensor pos, "
    "int window=0) -> Tensor",
    # attention-probability dropout regenerated from Philox(seed, offset) in the backward; `rng` is
    # the int64 [2] tensor {seed, offset} of the call (philox_rng: torch's generator, graph-safe)
    "flash_attn_fwd_drop(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens, int max_seqlen, float scale, bool causal, "
    "float p, Tensor rng) -> (Tensor, Tensor)",
    "flash_attn_bwd_drop(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor cu_seqlens, "
    "int max_seqlen, float scale, bool causal, float p, Tensor rng) -> (Tensor, Tensor, Tensor)",
    "flash_attn_bwd_qkv_drop(Tensor dout, Tensor qkv, int nq, int nkv, int head_dim, Tensor o, Tensor lse, "
    "Tensor cu_seqlens, int max_seqlen, float scale, bool causal, float p, Tensor rng) -> Tensor",
    "philox_rng(Tensor like, int increment) -> Tensor",
    "transpose2d(Tensor x) -> Tensor",
    # many matrices of a flat buffer transposed in one launch: rows of `mats` (int64 [n, 5]:
    # source offset, rows, cols, destination offset, first 64 x 64 tile); `mats_host` = its CPU copy
    "transpose_mats_(Tensor x, Tensor(a!) out, Tensor mats, Tensor mats_host, int ntiles) -> ()",
    "embedding_bwd_(Tensor(a!) out, Tensor ids, Tensor dy) -> ()",
    # FlashAttention-2-style varlen with explicit per-sequence key ranges (disjoint), causal mask
    # bottom-right aligned: context parallelism's local query chunks over gathered key prefixes
    "flash_attn_varlen_fwd(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens_q, Tensor k_start, Tensor k_len, "
    "int max_seqlen_q, int max_seqlen_k, float scale, bool causal) -> (Tensor, Tensor)",
    "flash_attn_varlen_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor cu_seqlens_q, "
    "Tensor k_start, Tensor k_len, int max_seqlen_q, int max_seqlen_k, float scale, bool causal) "
    "-> (Tensor, Tensor, Tensor)",
    "flash_attn_fwd_stamped(Tensor q, Tensor k, Tensor v, Tensor cu_seqlens, int max_seqlen, float scale, "
    "bool causal) -> (Tensor, Tensor, Tensor)",
    # backward launch tuning (read once from DTG_FA_* at load): set (kv_split, kv_qb), a negative
    # value keeps a knob; returns the previous pair.  `like` picks the device's implementation.
    "flash_attn_tuning(Tensor like, int kv_split, int kv_qb) -> int[]",
]

for _d in _DEFS:
    LIB.define(_d)
