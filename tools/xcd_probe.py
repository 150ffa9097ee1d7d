"""Where do the workgroups of a launch on a CU-masked stream run? Launches 16,384 sleeping
one-wave blocks of a probe kernel that records XCC_ID and HW_ID (SE / SH / CU fields) and
prints, per mask, the distinct hardware CUs used per XCD and per (XCD, SE).
usage: python tools/xcd_probe.py   (needs tools/libxcdprobe.so: hipcc -shared -fPIC
--offload-arch=gfx950 tools/xcd_probe.hip -o tools/libxcdprobe.so)"""
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
import torch  # noqa: E402

from heybuddy import _native  # noqa: E402
from heybuddy.pipeline import cu_mask_words, train_cu_set  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libxcdprobe.so"))
lib.xcd_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
hbk = _native.lib()
dev = torch.device("cuda:0")
n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
B = 16384
out = torch.zeros(2 * B, dtype=torch.int32, device=dev)


def where(cus, tag):
    words = cu_mask_words(cus, n_cu)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    _native.check(hbk.hbk_stream_create_cu_mask(arr, len(words), ctypes.byref(h)))
    s = torch.cuda.ExternalStream(h.value, device=dev)
    out.zero_()
    torch.cuda.synchronize()
    assert lib.xcd_probe(ctypes.c_void_p(out.data_ptr()), B, 20, ctypes.c_void_p(h.value)) == 0
    s.synchronize()
    hw = set()
    for a, b in out.cpu().view(-1, 2).tolist():
        hw.add((a & 0xF, (b >> 13) & 7, (b >> 12) & 1, (b >> 8) & 0xF))  # (xcc, se, sh, cu)
    per_xcd = collections.Counter(x for x, _, _, _ in hw)
    per_se = collections.Counter((x, se, sh) for x, se, sh, _ in hw)
    x0 = sorted((se, sh, cu) for x, se, sh, cu in hw if x == 0)
    print(f"{tag:>24}: {len(cus):3d} bits -> {len(hw):3d} CUs; per XCD {dict(sorted(per_xcd.items()))}; "
          f"XCD 0 per (SE, SH) {dict(sorted((k[1:], v) for k, v in per_se.items() if k[0] == 0))}; "
          f"XCD 0 CUs {x0}", flush=True)
    hbk.hbk_stream_destroy(h)


where(list(range(n_cu)), "all")
for lo in (0, 8, 32, 64):
    where(list(range(lo, lo + 32)), f"bits {lo}-{lo + 31}")
where(list(range(0, 8)), "bits 0-7")
for layout in ("spread", "se-balanced", "packed-contig"):
    t = train_cu_set(n_cu, 64, layout=layout)
    where(t, layout + " train")
    where(sorted(set(range(n_cu)) - set(t)), layout + " feat")
t = train_cu_set(n_cu, 64, layout="se-whole")
where(t, "se-whole train")
where(sorted(set(range(n_cu)) - set(t)), "se-whole feat")
