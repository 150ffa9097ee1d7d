"""Per-CU streaming bandwidth (tuning aid, not a test): GB/s per workgroup
and in total, one 256-thread workgroup per CU, on the whole GPU and on a
stream masked to N CUs (heybuddy.pipeline), from HBM (distinct regions) and
from L2 (one shared 1 MB region).

  python tools/bw_probe.py --build      (here: compiles tools/libbwprobe.so)
  python tools/bw_probe.py [--cus=64]
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
LIB = os.path.join(ROOT, "tools", "libbwprobe.so")

if "--build" in sys.argv:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(ROOT, "tools", "bwprobe.hip"), "-o", LIB], check=True)
    print(LIB)
    sys.exit(0)

import torch  # noqa: E402


def run(n_cus):
    lib = ctypes.CDLL(LIB)
    lib.bw_run.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_all = torch.cuda.get_device_properties(0).multi_processor_count
    stream = torch.cuda.current_stream()
    keep = None
    if n_cus:
        from heybuddy.pipeline import masked_stream, train_cu_set
        keep = masked_stream(dev, train_cu_set(n_all, n_cus))
        stream = keep.stream
    blocks = n_cus or n_all
    per_wg = (4 << 20) // 16  # 4 MB per workgroup
    buf = torch.empty(blocks * per_wg * 4 + 16, dtype=torch.float32, device=dev).uniform_()
    out = torch.zeros(256, device=dev)
    for shared, region in ((0, blocks * per_wg), (1, (1 << 20) // 16)):
        for depth in (1, 4, 8, 16):
            for wgs in (1, 2, 4):
                nb = blocks * wgs
                pw = per_wg // wgs
                with torch.cuda.stream(stream):
                    for _ in range(2):
                        lib.bw_run(buf.data_ptr(), pw, shared, region, out.data_ptr(), nb, depth, stream.cuda_stream)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        lib.bw_run(buf.data_ptr(), pw, shared, region, out.data_ptr(), nb, depth, stream.cuda_stream)
                    e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 5
                tot = nb * pw * 16 / (ms * 1e-3) / 1e9
                print(f"cus={n_cus or n_all} {'L2 ' if shared else 'HBM'} depth={depth:2d} wg/cu={wgs}: "
                      f"{tot:8.1f} GB/s total, {tot / blocks:6.1f} GB/s per CU ({ms * 1e3:.1f} us)", flush=True)


if __name__ == "__main__":
    run(next((int(a[6:]) for a in sys.argv[1:] if a.startswith("--cus=")), 0))
