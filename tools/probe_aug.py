"""Dev probe: time hbk_augment (noise mix + IR reverb, p = 1) on N clips with HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.dataset.augmented import BatchAugmenter  # noqa: E402
from heybuddy.synthetic import impulse_responses, noise_bank, synthetic_clips  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
dev = torch.device("cuda", 0)
x = synthetic_clips(n, seed=1, device=dev)
aug = BatchAugmenter(noise_bank(64, seed=2, device=dev), impulse_responses(32, seed=3, device=dev), device=dev,
                     batch_size=128, background_noise_prob=1.0, reverb_prob=1.0)
out = torch.empty((n, 23040), dtype=torch.float32, device=dev)
for _ in range(2):
    aug(x, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 3
e0.record()
for _ in range(reps):
    aug(x, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"augment: {n} clips {ms:.3f} ms  {n / ms * 1e3:.3e} clips/s  {n * 276480 / ms / 1e6:.1f} GB/s "
      f"finite={bool(torch.isfinite(out).all())}")
