"""Dev probe: time hbk_tanh_distortion on N clips with HIP events."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch
from heybuddy.kernels import tanh_distortion
from heybuddy.synthetic import synthetic_clips
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
x = synthetic_clips(n, length=23040, seed=1, device="cuda")
out = torch.empty_like(x)
amt = (torch.rand(n) * 0.1 + 1e-4).cuda()
for _ in range(2):
    tanh_distortion(x, amt, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
e0.record()
for _ in range(reps):
    tanh_distortion(x, amt, out=out)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
bytes_ = n * 23040 * 4 * 2
print(f"tanh: {n} clips {ms:.3f} ms  {n/ms*1e3:.3e} clips/s  {bytes_/ms/1e6:.1f} GB/s (x read + y written)")
