"""LDS bank-conflict model of the SoA mel kernel's accesses (mel_frames_soa_kernel, hbk_mel.hip).

Counts LDS-array cycles per processed group of one wave with the per-instruction lane groups
and bank functions of /opt/skills guides' MI355X LDS table (ds_read_b32 / ds_write_b32 /
ds_read2_b32 / ds_write2_b32: 2 x 32 lanes, bank (a/4) mod 32; ds_read2_b64: two accesses,
4 x 16 contiguous lanes, mod 32). Lane l works on frame f = l >> 3, column pair jj = l & 7.
usage: python tools/lds_bank_sim.py   (prints the kernel's layout against the r05 577-dword one)
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]
G32 = [range(0, 32), range(32, 64)]
G16 = [range(i, i + 16) for i in range(0, 64, 16)]


def cycles(addrs, groups, nb=32):
    tot = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for l in g:
            banks[addrs[l] % nb].add(addrs[l])
        tot += max(len(v) for v in banks.values())
    return tot


def layout_cost(fs, ld, pl, row, rows_b, po, lo):
    c = collections.Counter()

    def acc(name, fn, groups):
        c[name] += cycles([fn(l >> 3, l & 7) for l in range(64)], groups)

    for k1 in range(16):
        for off in (0, 8, pl, pl + 8):
            acc("stage-A stores", lambda f, jj: f * fs + row(k1) * ld + jj + off, G32)
    for n2 in range(16):
        for off in (0, pl):
            for r in (0, 1):
                acc("stage-B reads", lambda f, jj: f * fs + rows_b(jj)[r] * ld + n2 + off, G32)
    for k2 in range(8):
        acc("power stores", lambda f, jj: f * fs + po(f) + (jj if jj else 0) + 16 * k2, G32)
        acc("power stores", lambda f, jj: f * fs + po(f) + (16 - jj if jj else 8) + 16 * k2, G32)
    for idx, taps in ((0, 8), (8, 8), (16, 16), (24, 16)):
        for q in range(taps // 2):
            acc("filter reads", lambda f, jj: f * fs + po(f) + lo[idx + jj] + 2 * q, G16)
    return dict(c), sum(c.values())


def main():
    import numpy as np
    from oracle import mel as omel
    fb = np.asarray(omel.mel_fbank())
    if fb.shape[0] != 32:
        fb = fb.T
    lo = [int(np.nonzero(fb[m])[0][0]) & ~1 for m in range(32)]
    row4 = lambda k: 0 if k == 0 else 1 if k == 8 else 2 * k if k < 8 else 2 * (16 - k) + 1
    row5 = lambda k: 0 if k == 0 else 8 if k == 8 else k if k < 8 else 16 - k + 8
    old = layout_cost(577, 18, 288, row4, lambda jj: (2 * jj, 2 * jj + 1), lambda f: f & 1, lo)
    # one plane at a time through a 280-dword buffer: pl = 0 (each plane's accesses counted, as the kernel issues them)
    new = layout_cost(280, 17, 0, row5, lambda jj: (jj, jj + 8), lambda f: 24 * (f & 1) + 8 * ((f >> 1) & 1), lo)
    print("first 577-dword layout:", old)
    print("kernel layout (280):   ", new)


if __name__ == "__main__":
    main()
