"""Which XCDs / CUs do the workgroups of a launch on a CU-masked stream run on? For each
train-CU layout (heybuddy.pipeline.train_cu_set) and its complement, launch 1,024 one-wave
blocks of a probe kernel that records the XCC_ID and HW_ID registers, and print the
histogram of XCDs and the number of distinct CUs.
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
B = 1024
out = torch.zeros(2 * B, dtype=torch.int32, device=dev)


def probe(cus, tag):
    words = cu_mask_words(cus, n_cu)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    _native.check(hbk.hbk_stream_create_cu_mask(arr, len(words), ctypes.byref(h)))
    s = torch.cuda.ExternalStream(h.value, device=dev)
    out.zero_()
    torch.cuda.synchronize()
    assert lib.xcd_probe(ctypes.c_void_p(out.data_ptr()), B, 200, ctypes.c_void_p(h.value)) == 0
    s.synchronize()
    v = out.cpu().view(-1, 2).tolist()
    xh = collections.Counter(a & 0xF for a, _ in v)
    cus_seen = {(a & 0xF, b & 0xFFFF) for a, b in v}
    print(f"{tag:>26}: {len(cus)} mask bits -> XCD histogram {dict(sorted(xh.items()))}, "
          f"{len(cus_seen)} distinct (XCD, HW_ID) slots", flush=True)
    hbk.hbk_stream_destroy(h)


for layout in ("spread", "packed-rr", "packed-contig"):
    t = train_cu_set(n_cu, 64, layout=layout)
    probe(t, layout + " train")
    probe(sorted(set(range(n_cu)) - set(t)), layout + " featurize")
probe(list(range(n_cu)), "all")
probe(list(range(32)), "bits 0-31")
probe(list(range(0, n_cu, 8)), "bits 0, 8, 16, ...")
