"""Debug: FSDP + CPU offload (+AC) on one GPU, phase by phase with syncs and timestamps."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch

import dtg  # noqa: F401
from dtg.models import build_model, resolve_config
from dtg.parallel.checkpointing import apply_activation_checkpointing
from dtg.parallel.data_parallel import FlatAdamW
from dtg.parallel.fsdp import FullyShard

T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", flush=True)


name = sys.argv[1] if len(sys.argv) > 1 else "llama-3.1-8b"
dev = torch.device("cuda")
cfg = resolve_config(name)
model = build_model(cfg, device="meta", init=False)
log("meta model built")
eng = FullyShard(model, device=dev, cpu_offload=True)
log("engine constructed")
torch.cuda.synchronize()
log("synced after engine")
apply_activation_checkpointing(model)
opt = FlatAdamW(eng, lr=3e-5)
ids = torch.randint(0, cfg.vocab_size, (1, 4096), device=dev)
for step in range(2):
    opt.zero_grad()
    out = model(input_ids=ids, labels=ids)
    torch.cuda.synchronize()
    log(f"step {step} forward loss {out.loss.item():.3f}")
    eng.backward(out.loss)
    torch.cuda.synchronize()
    log(f"step {step} backward")
    opt.step()
    torch.cuda.synchronize()
    log(f"step {step} update")
