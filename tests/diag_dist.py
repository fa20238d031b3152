"""Diagnostic (GPU box): can a torchrun rank create a libsiftgpu context after the gloo rendezvous?"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
import sgpu  # noqa: E402

rank = int(os.environ.get("RANK", "0"))
env = {k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith("HIP") or k.startswith("ROC")}
print(rank, "env", env, flush=True)
sgpu.lib()
print(rank, "count before torch", sgpu.device_count(), flush=True)
import torch.distributed as dist  # noqa: E402
print(rank, "count after import", sgpu.device_count(), flush=True)
dist.init_process_group("gloo")
print(rank, "count after init", sgpu.device_count(), flush=True)
try:
    ctx = sgpu.SiftContext(0, sgpu.default_options())
    print(rank, "ctx ok", flush=True)
    ctx.close()
except Exception as e:
    print(rank, "ctx failed", e, flush=True)
dist.destroy_process_group()
