"""Dev probe: time hbk_augment (noise mix + IR reverb, p = 1) on N clips with HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
if "--phase" in sys.argv:  # profiling build: per-phase s_memtime cycles of augment_kernel
    sys.argv.remove("--phase")
    os.environ["HBK_LIB"] = os.path.join(ROOT, "hey-buddy_amd", "lib", "libhbk_phase.so")
import torch  # noqa: E402

from heybuddy.dataset.augmented import BatchAugmenter  # noqa: E402
from heybuddy.synthetic import impulse_responses, noise_bank, synthetic_clips  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
dev = torch.device("cuda", 0)
x = synthetic_clips(n, seed=1, device=dev)
aug = BatchAugmenter(noise_bank(64, seed=2, device=dev), impulse_responses(32, seed=3, device=dev), device=dev,
                     batch_size=128, background_noise_prob=1.0, reverb_prob=1.0, pitch_shift_prob=0.0)
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
if os.environ.get("HBK_LIB", "").endswith("libhbk_phase.so"):
    import ctypes
    from heybuddy._native import lib
    buf = (ctypes.c_ulonglong * 32)()
    fn = lib().hbk_debug_aug_phase
    fn.argtypes = [ctypes.c_void_p]
    fn(buf)  # reset
    aug(x, out=out)
    torch.cuda.synchronize()
    fn(buf)
    names = ["x->LDS", "noise E", "Ex/En sums", "mix", "a_in", "fwd16a", "fwd16b", "fwd9", "fwd5", "split*H",
             "inv5", "inv9", "inv16b", "inv16a", "a_out", "store"]
    tot = sum(buf[i] for i in range(16))
    print("phases: " + " ".join(f"{names[i]}={buf[i] / tot * 100:.1f}%" for i in range(16))
          + f"  total {tot / 1e6:.1f} Mcyc, {tot / n:.0f} cyc/clip (thread 0 of each block)", flush=True)
