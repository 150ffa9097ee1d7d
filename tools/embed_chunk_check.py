"""Embedding of N clips (SE20, split-f16) in one process with the chunk size in HBK_EMBED_CHUNK:
prints the time per call and a checksum of the output bits (chunking must not change them).
usage: HBK_EMBED_CHUNK=C python tools/embed_chunk_check.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.embedding_graph import WINDOW_STARTS, se20_graph  # noqa: E402
from heybuddy.kernels import EmbedPlan  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
g = torch.Generator(device="cuda").manual_seed(0)
mel = (torch.randn((n, 141, 32), device="cuda", generator=g) * 2 + 1).contiguous()
plan = EmbedPlan(se20_graph(), starts=WINDOW_STARTS, device=0, precision="split")
out = plan.clips(mel)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    out = plan.clips(mel)
e1.record()
torch.cuda.synchronize()
bits = out.contiguous().view(torch.int32).to(torch.int64)
print(f"chunk {os.environ.get('HBK_EMBED_CHUNK', 'default')}: {e0.elapsed_time(e1) / 3:.3f} ms per {n} clips; "
      f"checksum {int(bits.sum())} {int((bits * torch.arange(bits.numel(), device='cuda').view(bits.shape) % 1000003).sum())}",
      flush=True)
