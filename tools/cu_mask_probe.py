"""Does a CU mask restrict where a launch runs? Times a launch of many sleeping one-wave
blocks (tools/libxcdprobe.so, spin > 0) on streams masked to different CU sets: when the
mask is honoured the time grows as 256 / |mask|.
usage: python tools/cu_mask_probe.py"""
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


def timed(cus, tag):
    words = cu_mask_words(cus, n_cu)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    _native.check(hbk.hbk_stream_create_cu_mask(arr, len(words), ctypes.byref(h)))
    s = torch.cuda.ExternalStream(h.value, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        lib.xcd_probe(ctypes.c_void_p(out.data_ptr()), B, 50, ctypes.c_void_p(h.value))  # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            assert lib.xcd_probe(ctypes.c_void_p(out.data_ptr()), B, 50, ctypes.c_void_p(h.value)) == 0
        e1.record(s)
    s.synchronize()
    print(f"{tag:>28}: {len(cus):3d} mask bits  {e0.elapsed_time(e1) / 3 * 1e3:9.1f} us per launch", flush=True)
    hbk.hbk_stream_destroy(h)


timed(list(range(n_cu)), "all")
for layout in ("spread", "packed-rr", "packed-contig"):
    t = train_cu_set(n_cu, 64, layout=layout)
    timed(t, layout + " train (64)")
    timed(sorted(set(range(n_cu)) - set(t)), layout + " featurize (192)")
timed(list(range(32)), "bits 0-31")
timed(list(range(0, n_cu, 8)), "bits 0, 8, 16, ...")
timed(list(range(128)), "bits 0-127")
timed(list(range(0, n_cu, 2)), "even bits")
