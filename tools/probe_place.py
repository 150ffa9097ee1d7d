"""Dev probe: time hbk_place_clips on N synthetic utterances (0.3-1.5 s) placed to 23,040 samples."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from heybuddy.kernels import place_clips  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
rng = np.random.default_rng(0)
lens = rng.integers(4800, 24000, n).astype(np.int32)
pre = np.where(lens < 23040, rng.integers(0, 23040 - lens.clip(max=23039)), 0).astype(np.int32)
src = torch.randn((n, 24000), device="cuda")
ld, pd = torch.from_numpy(lens), torch.from_numpy(pre)
out = place_clips(src, lens, pre, 23040)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    out = place_clips(src, lens, pre, 23040)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
gb = (lens.clip(max=23040).sum() * 4 + n * 23040 * 4) / 1e9
print(f"place: {n} clips {ms:.3f} ms  {gb / ms:.2f} TB/s algorithmic ({gb:.2f} GB)")
