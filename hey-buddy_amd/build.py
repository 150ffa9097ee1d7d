"""Build libhbk.so (all HIP kernels + the C ABI) for gfx950, in-tree.

Usage: python hey-buddy_amd/build.py [--force]
The library lands in hey-buddy_amd/lib/libhbk.so, next to the Python package
that loads it, so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libhbk.so")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-I", INCLUDE, "-I", CSRC, "-Wall", "-Wno-unused-function",
    "-munsafe-fp-atomics",
]
# Per-file flags. hbk_mel.hip: no SLP vectorisation of scalar f32 code (it packs
# the mel dot products into v_pk_fma_f32 plus register moves; the complex
# arithmetic there is already explicit float2 vector code).
FILE_FLAGS = {"hbk_mel.hip": ("-fno-slp-vectorize",)}


def sources() -> list[str]:
    return sorted(
        os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp"))
    )


def _headers_mtime() -> float:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src: str, force: bool, obj_dir: str = OBJ, extra: tuple = ()) -> str:
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime()):
            return obj
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(os.path.basename(src), ()), *extra, *lang, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


VARIANTS = {  # profiling builds (load with HBK_LIB=hey-buddy_amd/lib/<name>)
    "phase": ("libhbk_phase.so", ("-DHBK_PHASE_TIMING",)),  # s_memtime phase counters + ablation
    "ablate": ("libhbk_ablate.so", ("-DHBK_ABLATE",)),      # HBK_DEBUG_SKIP phase ablation only
    "trace": ("libhbk_trace.so", ("-DHBK_TRACE",)),         # per-wave s_memtime timeline
    "pv32": ("libhbk_pv32.so", ("-DHBK_PV_F32STATE=1",)),  # the vocoder's sliding-DFT state in float32
    "pv32r": ("libhbk_pv32r.so", ("-DHBK_PV_F32STATE=1", "-DHBK_PV_RESTART=1024")),  # ... restarted every 1,024
}
# Any other ablation / A/B build: --variant=NAME --define=MACRO[=VALUE] ... (e.g. --variant=kvab1
# --define=HBK_KV_ABLATE=1 -> lib/libhbk_kvab1.so; the macros are documented where they are used:
# HBK_K2_ABLATE, HBK_KV_ABLATE, HBK_PV_ABLATE, HBK_PV_CLIPS, HBK_PV_RESTART, HBK_X3_WAVES_PER_EU, HBK_X3_PF)


def build(force: bool = False, variant: str | None = None) -> str:
    obj_dir = OBJ + (f"_{variant}" if variant else "")
    lib = os.path.join(LIB_DIR, VARIANTS[variant][0]) if variant else LIB
    extra = VARIANTS[variant][1] if variant else ()
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, obj_dir, extra), srcs))
    if (not force and os.path.exists(lib)
            and os.path.getmtime(lib) >= max(os.path.getmtime(o) for o in objs)):
        return lib
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    var = next((a[len("--variant="):] for a in sys.argv if a.startswith("--variant=")), None)
    defs = tuple("-D" + a[len("--define="):] for a in sys.argv if a.startswith("--define="))
    if var and defs:
        VARIANTS[var] = (f"libhbk_{var}.so", defs)
    elif var and var not in VARIANTS:
        sys.exit(f"unknown variant {var!r}: pass its macros with --define=MACRO[=VALUE]")
    print(build(force="--force" in sys.argv, variant=var))
