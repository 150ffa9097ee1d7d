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
if "--phase" in sys.argv:
    os.environ["HBK_LIB"] = os.path.join(ROOT, "hey-buddy_amd", "lib", "libhbk_phase.so")
if "--lib" in sys.argv:  # A/B against another build: prototypes it does not export are dropped
    os.environ["HBK_LIB"] = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])

import torch  # noqa: E402

from heybuddy.embedding_graph import WINDOW_STARTS, se20_graph  # noqa: E402
from heybuddy.kernels import EmbedPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--precision", default="both")
    ap.add_argument("--lib", default=None, help="load this libhbk build instead (A/B timing)")
    ap.add_argument("--phase", action="store_true",
                    help="load lib/libhbk_phase.so and print per-chain phase cycles (wave 0 of each block)")
    a = ap.parse_args()
    if a.lib:
        import ctypes
        from heybuddy import _native
        h = ctypes.CDLL(os.environ["HBK_LIB"])
        for name in [n for n in _native._PROTOS if not hasattr(h, n)]:
            _native._PROTOS.pop(name)
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
        if a.phase and p == "split":
            import ctypes
            from heybuddy._native import lib
            buf = (ctypes.c_ulonglong * 64)()
            fn = lib().hbk_debug_phase_cycles
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
            fn(buf, 64)  # reset after the timed loop
            plan.clips(mel)
            torch.cuda.synchronize()
            fn(buf, 64)
            for ch in range(4):
                row = [buf[ch * 16 + i] for i in range(16)]
                tot = sum(row)
                if tot:
                    print(f"chain {ch}: " + " ".join(f"p{i}={v / tot * 100:.1f}%" for i, v in enumerate(row) if v)
                          + f"  total {tot / 1e6:.1f} Mcyc (sum over blocks, wave 0)", flush=True)


if __name__ == "__main__":
    main()
