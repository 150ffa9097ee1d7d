#!/usr/bin/env python
"""bench.py — the BASELINE.json metric on the MI355X hot path.

Metric: audio clips/sec featurized (1.5 s @ 16 kHz synthetic clips), at N GPUs.
Workload (BASELINE.json configs[1]): per rank, 100 k clips resident in HBM are
featurized exactly as SpeechEmbeddings.__call__ does (reference
embeddings.py:153-234): STFT + 32-bin log-mel (hbk_mel_frames), the speech
embedding graph on the 16 reference windows per clip (hbk_embed_clips, the
SE20 stand-in graph — the real ONNX graph is absent offline), NaN-row
replacement. One step = one pass over the 100 k clips.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL). Featurization shards the
clips with no data-path collective ("weak" scaling: every rank featurizes its
own 100 k clips); the timed region is bracketed by barrier + synchronize and
the max over ranks is reported.

rank 0 prints ONE JSON line with the metric, a ``roofline`` object for the
dominant kernel (measured live with HIP events on the stream the kernels run
on), a ``roofline_mel`` object for the STFT+mel kernel, and a ``cpu_baseline``
(the oracle's CPU featurizer on a bounded sample, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hey-buddy_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense f32 MFMA = f32 vector peak
MEL_READ_SAMPLES = 22912     # frame 140 ends at 140*160 + 512
N_FRAMES = 141


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--clips", type=int, default=100_000, help="clips per rank per step")
    ap.add_argument("--cpu-sample", type=int, default=3000, help="clips timed on the host CPU (~10-30 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r01.json"),
                    help="per-kernel HBM bytes from a rocprofv3 --pmc pass (optional)")
    return ap.parse_args()


def load_traffic(path, kernel_substr, launches_per_step):
    try:
        with open(path) as f:
            d = json.load(f)
        for name, v in d.get("kernels", {}).items():
            if kernel_substr in name:
                return v.get("hbm_bytes_per_step", v.get("hbm_bytes_per_launch", 0) * launches_per_step)
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from heybuddy.embeddings import SpeechEmbeddings, _replace_nan_rows, embed_plan
    from heybuddy.embedding_graph import WINDOW_STARTS
    from heybuddy.kernels import embed_clips, mel_frames
    from heybuddy.spectrogram import default_mel_plan
    from heybuddy.synthetic import seed_for, synthetic_clips

    n = args.clips
    clips = synthetic_clips(n, seed=seed_for(2, rank), device=dev)
    se = SpeechEmbeddings(device_id=local)
    mplan = default_mel_plan(dev, 32767.0)
    eplan = embed_plan(dev, WINDOW_STARTS)
    stream = torch.cuda.current_stream(dev)

    def step(evs=None):
        if evs:
            evs[0].record(stream)
        frames = mel_frames(clips, mplan, N_FRAMES)
        if evs:
            evs[1].record(stream)
        emb = embed_clips(frames, eplan)
        if evs:
            evs[2].record(stream)
        return _replace_nan_rows(emb)

    # the step is SpeechEmbeddings.featurize; check once that they agree
    ref = se.featurize(clips[:64])
    got = step()[:64]
    assert torch.equal(ref, got), "bench step diverges from SpeechEmbeddings.featurize"

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    mel_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    emb_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    mel_bytes = n * (MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4)
    emb_flops = 2.0 * eplan.macs_per_clip * n
    mel_gbs = mel_bytes / (mel_ms * 1e-3) / 1e9
    emb_tf = emb_flops / (emb_ms * 1e-3) / 1e12
    roof_emb = {
        "kernel": "conv_chain_kernel (hbk_embed_clips: %d chained launches per %d-clip chunk)"
                  % (eplan.n_chains, min(n, 16384)),
        "bound": "mfma", "achieved": round(emb_tf, 3), "peak": FP32_MFMA_PEAK_TFLOPS,
        "unit": "TFLOP/s", "frac": round(emb_tf / FP32_MFMA_PEAK_TFLOPS, 4),
        "traffic": load_traffic(args.pmc, "conv_chain", 1),
        "algorithmic_flops_per_clip": 2.0 * eplan.macs_per_clip, "ms_per_step": round(emb_ms, 3),
    }
    roof_mel = {
        "kernel": "mel_frames_kernel (hbk_mel_frames, 1 launch per step)",
        "bound": "hbm", "achieved": round(mel_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(mel_gbs / HBM_PEAK_GBS, 4),
        "traffic": load_traffic(args.pmc, "mel_frames", 1),
        "algorithmic_bytes_per_clip": MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4,
        "ms_per_step": round(mel_ms, 3),
    }
    dominant, other = (roof_emb, roof_mel) if emb_ms >= mel_ms else (roof_mel, roof_emb)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        import numpy as np
        from heybuddy.embeddings import default_graph
        from oracle.featurizer import cpu_featurize
        threads = min(16, os.cpu_count() or 1)
        sample = clips[:args.cpu_sample].cpu().numpy()
        cpu_featurize(sample[:4], default_graph(), threads=threads)  # warm
        c0 = time.perf_counter()
        cpu_featurize(sample, default_graph(), threads=threads)
        c_el = time.perf_counter() - c0
        cpu = {"value": round(args.cpu_sample / c_el, 2), "unit": "clips/s", "cores": threads,
               "kind": "port",
               "sample": f"{args.cpu_sample} of the step's clips through oracle/featurizer.cpu_featurize "
                         f"(reference cost structure: 4x105 mel frames + 16 windows/clip, batch 64; "
                         f"numpy fp32 FFT + torch CPU fp32 conv), {c_el:.1f} s"}

    if rank == 0:
        value = world * n * args.steps / elapsed
        line = {
            "metric": "audio clips/sec featurized+trained, 1.5 s @16 kHz, 1/2/4/8 GPU",
            "value": round(value, 1), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic 1.5 s @16 kHz clips (seeded), SE20 stand-in embedding graph",
            "config": {"workload": "configs[1]: 100k clips mel-STFT + speech-embedding forward per GPU",
                       "clips_per_rank": n, "clip_samples": int(clips.shape[1]),
                       "mel_frames_per_clip": N_FRAMES, "windows_per_clip": len(WINDOW_STARTS),
                       "parallelism": f"dp{world} (clip shards, no collective)"},
            "roofline": dominant, "roofline_other": other, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
