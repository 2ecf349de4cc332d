"""MI355X-native distributed causal-LM training framework (import name: `dtg`).

Capabilities mirror rimelabs/lambda-labs_distributed-training-guide:
single-GPU -> DDP/ZeRO -> FSDP -> 405B -> tensor/sequence parallel -> 2-D parallel,
with hand-written gfx950 HIP kernels on the hot path (`dtg.ops`), owned Llama/GPT-2
models (`dtg.models`), RCCL-based parallel engines (`dtg.parallel`) and the training
driver, checkpointing and observability (`dtg.train`, `dtg.utils`).
"""
__version__ = "0.1.0"
