"""Time hbk_pitch_shift on a batch of clips (HIP events on the current stream).
usage: python tools/probe_pitch.py [n_clips] [iters]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..",
                                                                             "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy.kernels import pitch_shift  # noqa: E402
from heybuddy.synthetic import synthetic_clips  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
x = synthetic_clips(n, length=23040, seed=3).cuda()
idx = torch.arange(n, dtype=torch.int32, device="cuda")
for num, den in ((128, 125), (125, 128)):
    pitch_shift(x, idx, num, den, out=x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        pitch_shift(x, idx, num, den, out=x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"pitch {num}/{den}: {n} clips {ms:.3f} ms -> {ms * 1e3 / n:.2f} us/clip", flush=True)
    if os.environ.get("HBK_LIB", "").endswith("libhbk_phase.so"):  # vocoder phase cycles (wave 0 per block)
        import ctypes
        from heybuddy._native import lib
        buf = (ctypes.c_ulonglong * 32)()
        fn = lib().hbk_debug_aug_phase
        fn.argtypes = [ctypes.c_void_p]
        fn(buf)
        pitch_shift(x, idx, num, den, out=x)
        torch.cuda.synchronize()
        fn(buf)
        names = ["init", "refill", "frames", "G->LDS+barrier", "istft"]
        tot = sum(buf[16 + i] for i in range(5))
        blocks = (n + 1) // 2  # HBK_PV_CLIPS (2)
        print("  vocoder phases: " + " ".join(f"{names[i]}={buf[16 + i] / tot * 100:.1f}%" for i in range(5))
              + f"  {tot / blocks:.0f} cyc/block (wave 0)", flush=True)
