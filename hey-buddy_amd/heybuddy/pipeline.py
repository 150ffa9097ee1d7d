"""Overlapping featurization with classifier training on one GPU.

The reference runs the two phases of ``heybuddy train`` one after the other:
every clip is augmented and featurized first, then the classifier trains on
the stored features (__main__.py:245-429, features.py:492-535,
trainer.py:764-1007). On MI355X the train step at the reference's batch of
1,100 rows is a latency-bound chain that fills a fraction of the 256 CUs
(k2 runs one workgroup per 16-row tile: 69 workgroups), while featurization is
throughput work that fills any CU it is given. So the pipelined driver trains
on chunk s while chunk s + 1 is augmented and featurized beside it, on a
second stream, with two embedding pools:

  feature stream:  featurize(s + 1) -> pool[(s + 1) % 2]   (waits train(s - 1))
  train stream:    train(s) on pool[s % 2]                 (waits featurize(s))

The work is the same as the sequential order (every clip featurized once and
trained on once, the model updated in the same step order); only the
placement in time changes. How the two streams share the CUs is a policy:

  "prio"       both streams on the whole device, the train stream at high
               priority (the dispatcher prefers its waiting workgroups);
  "split:N"    the train stream on N CUs of its own, featurization on the rest
               (hipExtStreamCreateWithCUMask, hbk_stream_create_cu_mask);
  "spill:N"    featurization on all but N CUs, the train stream on the whole
               device at high priority (its wide launches spill into the
               featurization CUs as their workgroups retire).
"""
from __future__ import annotations

import atexit
import ctypes
from typing import List, Optional, Tuple

import torch

__all__ = ["train_cu_set", "cu_mask_words", "masked_stream", "make_streams"]


def train_cu_set(n_cu: int, n_train: int, n_xcd: int = 8, layout: Optional[str] = None) -> List[int]:
    """The train partition's CU ids (mask bits). "spread" (default): n_train ids
    spread evenly over the XCDs whether the mask's bit i maps to XCD
    i // (n_cu / n_xcd) or to XCD i % n_xcd: XCD x takes the k = n_train / n_xcd
    ids x * per + (floor(j per / k) + x) mod per (per = CUs per XCD).
    "packed-rr" / "packed-contig": whole XCDs (n_train / per of them), for bit i
    on XCD i % n_xcd / i // per (HBK_TRAIN_CU_LAYOUT; tools/xcd_probe.py maps the
    bits on a device)."""
    import os
    layout = layout or os.environ.get("HBK_TRAIN_CU_LAYOUT", "spread")
    per = n_cu // n_xcd
    if layout == "se-whole":  # whole shader engines: mask bit i = XCD i % 8, SE (i // 8) % 4, CU i // 32 (probed)
        n_se = 4
        per_se = n_cu // (n_xcd * n_se)
        if n_train % (n_xcd * per_se) == 0:
            ses = n_train // (n_xcd * per_se)
            return sorted(i for i in range(n_cu) if (i // n_xcd) % n_se < ses)
    if layout == "se-balanced" and n_train % n_xcd == 0:  # every XCD, and within it every quarter of its CUs
        k = n_train // n_xcd                              # (bit i: XCD i % n_xcd, CU i // n_xcd)
        if k % 4 == 0:
            q = per // 4
            return sorted(x + n_xcd * (s_ * q + j) for x in range(n_xcd) for s_ in range(4) for j in range(k // 4))
    if layout.startswith("xcds-rr:"):  # n_train CUs on the first X XCDs (bit i on XCD i % n_xcd), n_train / X each
        nx = int(layout.split(":")[1])
        if 0 < nx <= n_xcd and n_train % nx == 0 and n_train // nx <= per:
            return sorted(x + n_xcd * j for x in range(nx) for j in range(n_train // nx))
    if layout in ("packed-rr", "packed-contig") and n_train % per == 0:
        xcds = range(n_train // per)
        if layout == "packed-rr":
            return sorted(x + n_xcd * j for x in xcds for j in range(per))
        return sorted(x * per + j for x in xcds for j in range(per))
    k = max(1, min(per, n_train // n_xcd))
    return sorted(x * per + ((j * per // k + x) % per) for x in range(n_xcd) for j in range(k))


def cu_mask_words(cus, n_cu: int) -> List[int]:
    words = [0] * ((n_cu + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    return words


class _MaskedStream:
    """A hipExtStreamCreateWithCUMask stream wrapped as a torch ExternalStream
    (destroyed with this object)."""

    def __init__(self, device: torch.device, cus):
        from . import _native
        self._lib = _native.lib()
        n_cu = torch.cuda.get_device_properties(device).multi_processor_count
        words = cu_mask_words(cus, n_cu)
        arr = (ctypes.c_uint32 * len(words))(*words)
        handle = ctypes.c_void_p()
        with torch.cuda.device(device):
            _native.check(self._lib.hbk_stream_create_cu_mask(arr, len(words), ctypes.byref(handle)))
        self.handle = handle
        self.stream = torch.cuda.ExternalStream(handle.value, device=device)
        self.cus = list(cus)
        self.device = device
        _MASKS[handle.value] = self.cus
        _LIVE[id(self)] = self
        _register_teardown()

    def destroy(self) -> None:
        """Synchronise and destroy the stream (idempotent). Called by __del__
        while the interpreter runs, and for every live stream by the atexit hook
        (_teardown), i.e. while the HIP runtime is still up: a hipStreamDestroy
        left to module teardown ran after the runtime (and rocprofv3's tool
        library) had begun shutting down and crashed in __cxa_finalize."""
        h, self.handle = self.handle, None
        _LIVE.pop(id(self), None)
        if not h or not h.value or _SHUTDOWN[0]:
            return
        _MASKS.pop(h.value, None)
        self.stream.synchronize()  # this stream only: no device-wide stall
        self._lib.hbk_stream_destroy(h)

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


_MASKS: dict = {}  # raw stream handle -> its CU set (the live _MaskedStreams)
_CAPTURE: dict = {}  # (device, CU set) -> the one masked capture stream kept for it
_LIVE: dict = {}  # id -> every _MaskedStream not yet destroyed
_SHUTDOWN = [False]
_REGISTERED = [False]


def _teardown() -> None:
    """atexit: drain the device, then destroy every live masked stream while the
    HIP runtime is alive; later __del__ calls (module teardown) do nothing."""
    try:
        if _LIVE:
            torch.cuda.synchronize()
        _CAPTURE.clear()
        for ms in list(_LIVE.values()):
            try:
                ms.destroy()
            except Exception:
                pass
    finally:
        _SHUTDOWN[0] = True


def _register_teardown() -> None:
    # registered at the first masked stream, i.e. after torch's own atexit
    # hooks, so it runs before them (atexit is LIFO)
    if not _REGISTERED[0]:
        _REGISTERED[0] = True
        atexit.register(_teardown)


def masked_stream(device: torch.device, cus) -> "_MaskedStream":
    return _MaskedStream(device, cus)


def capture_stream(device: torch.device):
    """A side stream for capturing work that will replay on the current
    stream: with the current stream's CU mask if it has one, so that kernels
    sizing their grids (or picking a variant) by the stream's CUs at capture
    time see the CUs they will replay on. Returns (stream, keep-alive)."""
    cur = torch.cuda.current_stream(device)
    cus = _MASKS.get(cur.cuda_stream)
    if cus is None:
        return torch.cuda.Stream(device), None
    key = (str(device), tuple(cus))
    ms = _CAPTURE.get(key)  # one per CU set, reused: no stream create / destroy per capture
    if ms is None:
        ms = _CAPTURE[key] = _MaskedStream(device, cus)
    return ms.stream, ms


def make_streams(device: torch.device, policy: str) -> Tuple[torch.cuda.Stream, torch.cuda.Stream, list]:
    """(feature stream, train stream, keep-alive objects) for a policy string
    ("prio", "split:N", "spill:N")."""
    n_cu = torch.cuda.get_device_properties(device).multi_processor_count
    keep: list = []
    if policy == "prio":
        return torch.cuda.Stream(device), torch.cuda.Stream(device, priority=-1), keep
    kind, _, n = policy.partition(":")
    n = int(n)
    if kind not in ("split", "spill") or not 0 < n < n_cu:
        raise ValueError(f"unknown overlap policy {policy!r}")
    train = train_cu_set(n_cu, n)
    feat = masked_stream(device, sorted(set(range(n_cu)) - set(train)))
    keep.append(feat)
    if kind == "split":
        ts = masked_stream(device, train)
        keep.append(ts)
        return feat.stream, ts.stream, keep
    return feat.stream, torch.cuda.Stream(device, priority=-1), keep
