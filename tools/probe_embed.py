"""Embedding chain probe: prints each chain's layout (HBK_DEBUG_EMBED) and times
hbk_embed_clips on one 16384-clip chunk per precision. Run under
``rocprofv3 --kernel-trace --stats -f csv`` for per-chain kernel times.

usage: python tools/probe_embed.py [--clips N] [--iters K] [--precision split|exact|both]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
os.environ.setdefault("HBK_DEBUG_EMBED", "1")

import torch  # noqa: E402

from heybuddy.embedding_graph import WINDOW_STARTS, se20_graph  # noqa: E402
from heybuddy.kernels import EmbedPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--precision", default="both")
    a = ap.parse_args()
    g = se20_graph()
    mel = (torch.randn((a.clips, 141, 32), device="cuda") * 2 + 1).contiguous()
    precs = ["split", "exact"] if a.precision == "both" else [a.precision]
    for p in precs:
        print(f"--- {p}", flush=True)
        plan = EmbedPlan(g, starts=WINDOW_STARTS, device=0, precision=p)
        out = plan.clips(mel)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            out = plan.clips(mel)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.iters
        tf = 2 * plan.macs_per_clip * a.clips / (ms * 1e-3) / 1e12
        print(f"{p}: {ms:.3f} ms per {a.clips} clips = {tf:.1f} TFLOP/s algorithmic, "
              f"finite={bool(torch.isfinite(out).all())}", flush=True)


if __name__ == "__main__":
    main()
