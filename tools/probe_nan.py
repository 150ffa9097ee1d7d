"""Dev probe: time the NaN-row replacement of a 100 k-clip embedding batch: in place
(hbk_nan_rows_fix) against the gather form (replace_nan_rows_device), on the whole GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.embeddings import replace_nan_rows_device  # noqa: E402
from heybuddy.kernels import nan_rows_fix  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
dev = torch.device("cuda", 0)
pool = torch.randn(n, 16, 96, device=dev)
ext = torch.zeros(n + 1, 16, 96, device=dev)
ext[:n] = pool
out = torch.empty_like(pool)
ws = torch.empty(2 * n * 4 + 64, dtype=torch.uint8, device=dev)


def timed(fn, tag):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per call", flush=True)


timed(lambda: nan_rows_fix(pool, seed=1, ws=ws), "in place (hbk_nan_rows_fix)")
timed(lambda: replace_nan_rows_device(ext, out=out, zero_row=True), "gather (replace_nan_rows_device)")
