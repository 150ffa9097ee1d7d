"""Per-wave s_memtime timeline of the first tasks of the first split chain
(lib/libhbk_trace.so; tuning aid). Marks: 1 task start, 19 pre-barrier,
20+s stage s start, 10 unit start, 11 prologue done, 12 k-loop done,
13 epilogue done, 5 store start, 6 task end."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
os.environ["HBK_LIB"] = os.path.join(ROOT, "hey-buddy_amd", "lib", "libhbk_trace.so")

import torch  # noqa: E402

from heybuddy._native import lib  # noqa: E402
from heybuddy.embedding_graph import WINDOW_STARTS, se20_graph  # noqa: E402
from heybuddy.kernels import EmbedPlan  # noqa: E402

NAMES = {1: "task", 19: "bar>", 5: "store", 6: "end", 10: "unit", 11: "pro", 12: "mma", 13: "epi",
         40: "raw|", 50: "s0>", 41: "s0|", 51: "s1>", 42: "s1|", 52: "s2>", 43: "s2|"}  # p0: > done, | after barrier


def main():
    clips = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    plan = EmbedPlan(se20_graph(), starts=WINDOW_STARTS, device=0, precision="split")
    mel = (torch.randn((clips, 141, 32), device="cuda") * 2 + 1).contiguous()
    fn = lib().hbk_debug_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * (16 * 256))()
    cnt = (ctypes.c_int * 16)()
    plan.clips(mel)
    torch.cuda.synchronize()
    fn(buf, cnt)  # reset
    plan.clips(mel)
    torch.cuda.synchronize()
    fn(buf, cnt)
    for b in range(2):
        t0 = min(buf[(b * 4 + w) * 256] >> 8 for w in range(4) if cnt[b * 4 + w])
        for w in range(4):
            n = cnt[b * 4 + w]
            ev = [(buf[(b * 4 + w) * 256 + i] >> 8, buf[(b * 4 + w) * 256 + i] & 255) for i in range(n)]
            line = []
            prev = t0
            for t, i in ev[:60]:
                nm = NAMES.get(i, f"s{i - 20}" if 20 <= i < 40 else str(i))
                line.append(f"{nm}+{(t - prev)}")
                prev = t
            print(f"block {b} wave {w} ({n} ev): " + " ".join(line))


if __name__ == "__main__":
    main()
