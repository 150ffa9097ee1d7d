#!/usr/bin/env python
"""bench.py — the BASELINE.json metric on the MI355X hot path.

Metric: audio clips/sec featurized (1.5 s @ 16 kHz synthetic clips), at N GPUs.

Workloads (BASELINE.json configs; --config, default 2 = configs[1]):
  2  per rank, 100 k clips resident in HBM are featurized exactly as
     SpeechEmbeddings.__call__ does (reference embeddings.py:153-234):
     STFT + 32-bin log-mel (hbk_mel_frames), the speech-embedding graph on the
     16 reference windows per clip (hbk_embed_clips; SE20 stand-in graph — the
     real ONNX graph is absent offline), NaN-row replacement.
  3  the same after on-device augmentation (configs[2]): background-noise mix
     + IR reverb with p forced to 1, one IR per 128-clip batch, and the
     reference's per-batch Gain (p 1.0 by default) (hbk_augment).
  4  classifier training (configs[3]): stage-1 steps at the reference's global
     batch of 1,100 embeddings (50 positive / 50 adversarial / 1,000 negative)
     sampled on the device; metric embeddings/s trained.
One step = one pass of the hot path over one batch (100 k clips; 1 train step).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL). Featurization shards the
clips with no data-path collective ("weak": every rank featurizes its own
100 k clips); training splits each global batch over the ranks with one
all-reduce of the gradient bucket per step ("strong"). The timed region is
bracketed by barrier + synchronize and the max over ranks is reported.

rank 0 prints ONE JSON line: the metric, ``roofline`` for the dominant kernel
(algorithmic work / its average duration, timed live with HIP events on the
stream the kernels run on), ``roofline_other`` for the other stages, and a
``cpu_baseline`` (the oracle's CPU path on a bounded sample, N = 1 only).
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

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense f32 MFMA = f32 vector peak
F16_MFMA_PEAK_TFLOPS = 2516.6  # dense f16 MFMA: 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz
# split-f16 embedding GEMMs issue 3 f16 products per f32-accurate MAC
SPLIT_PEAK_TFLOPS = round(F16_MFMA_PEAK_TFLOPS / 3, 1)
MEL_READ_SAMPLES = 22912       # frame 140 ends at 140*160 + 512
N_FRAMES = 141
AUG_T = 23040


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4))
    ap.add_argument("--clips", type=int, default=100_000, help="clips per rank per step (configs 2, 3)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="units timed on the host CPU (~10-30 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--full-augment", action="store_true",
                    help="config 3 plus the reference's tanh distortion and colored noise at their default "
                         "probabilities (0.25 each); not the BASELINE configs[2] workload")
    ap.add_argument("--no-check", action="store_true", help="skip the one-off featurize equality check")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="per-kernel HBM bytes from rocprofv3 --pmc passes (optional)")
    return ap.parse_args()


def load_traffic(path, kernel_substr):
    """HBM bytes per step of the kernels whose name contains kernel_substr (a
    string or a tuple of alternatives), from a tools/pmc_summary.py JSON
    (FETCH_SIZE doubled per the gfx950 calibration + WRITE_SIZE), or None."""
    subs = (kernel_substr,) if isinstance(kernel_substr, str) else tuple(kernel_substr)
    try:
        with open(path) as f:
            d = json.load(f)
        v = [k for name, k in d.get("kernels", {}).items() if any(s in name for s in subs)]
        if v:
            return sum(k["hbm_bytes_per_step"] for k in v)
    except (OSError, ValueError, KeyError):
        pass
    return None


def roof(kernel, bound, work, ms, unit, traffic, peak=None, **extra):
    ach = work / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
    if peak is None:
        peak = HBM_PEAK_GBS if unit == "GB/s" else FP32_MFMA_PEAK_TFLOPS
    d = {"kernel": kernel, "bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": unit,
         "frac": round(ach / peak, 4), "traffic": traffic, "ms_per_step": round(ms, 3)}
    d.update(extra)
    return d


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=dev)

    from heybuddy.synthetic import seed_for
    setup = {2: setup_featurize, 3: setup_featurize, 4: setup_train}[args.config]
    job = setup(args, dev, rank, world, seed_for(args.config, rank))
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        job["step"](None)
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(len(job["stages"]) + 1)]
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        job["step"](evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    stage_ms = [sum(e[i].elapsed_time(e[i + 1]) for e in evs) / args.steps for i in range(len(job["stages"]))]
    roofs = [job["roofline"](name, ms, args.pmc) for name, ms in zip(job["stages"], stage_ms)]
    dom = max(range(len(roofs)), key=lambda i: stage_ms[i])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = job["cpu_baseline"](args.cpu_sample)

    if rank == 0:
        units = job["units_per_step"] * (world if job["scaling"] == "weak" else 1)
        value = units * args.steps / elapsed
        line = {
            "metric": job["metric"], "value": round(value, 1), "unit": job["unit"], "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": job["scaling"], "vs_baseline": None, "dtype": "f32",
            "data": job["data"], "config": job["config"], "roofline": roofs[dom],
            "roofline_other": [r for i, r in enumerate(roofs) if i != dom], "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# --------------------------------------------------------- configs 2 / 3 ----
def setup_featurize(args, dev, rank, world, seed):
    from heybuddy.dataset.augmented import BatchAugmenter
    from heybuddy.embedding_graph import WINDOW_STARTS
    from heybuddy.embeddings import SpeechEmbeddings, _replace_nan_rows, default_graph, embed_plan
    from heybuddy.kernels import embed_clips, mel_frames
    from heybuddy.spectrogram import default_mel_plan
    from heybuddy.synthetic import impulse_responses, noise_bank, synthetic_clips

    n = args.clips
    augment = args.config == 3
    clips = synthetic_clips(n, seed=seed, device=dev)
    mplan = default_mel_plan(dev, 32767.0)
    eplan = embed_plan(dev, WINDOW_STARTS)
    aug = None
    if augment:
        aug = BatchAugmenter(noise_bank(64, seed=seed + 1, device=dev),
                             impulse_responses(32, seed=seed + 2, device=dev), device=dev, batch_size=128,
                             background_noise_prob=1.0, reverb_prob=1.0,
                             colored_noise_prob=0.25 if args.full_augment else 0.0,
                             tanh_distortion_prob=0.25 if args.full_augment else 0.0)  # configs[2]: reverb + noise (+ gain)
        aug_out = torch.empty((n, AUG_T), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    stages = (["augment"] if augment else []) + ["mel", "embed"]

    def step(evs):
        i = 0
        if evs:
            evs[i].record(stream)
        x = clips
        if augment:
            x = aug(clips, out=aug_out)
            i += 1
            if evs:
                evs[i].record(stream)
        frames = mel_frames(x, mplan, N_FRAMES)
        i += 1
        if evs:
            evs[i].record(stream)
        emb = embed_clips(frames, eplan)
        i += 1
        if evs:
            evs[i].record(stream)
        return _replace_nan_rows(emb)

    if not augment and not args.no_check:  # the step is SpeechEmbeddings.featurize; check once
        ref = SpeechEmbeddings(device_id=dev.index).featurize(clips[:64])
        assert torch.equal(ref, step(None)[:64]), "bench step diverges from SpeechEmbeddings.featurize"

    def roofline(name, ms, pmc):
        if name == "mel":
            return roof("mel_frames_v2_kernel (hbk_mel_frames, 1 launch per step)", "hbm",
                        n * (MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4), ms, "GB/s", load_traffic(pmc, "mel_frames"),
                        algorithmic_bytes_per_clip=MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4)
        if name == "embed":
            split = eplan.precision == "split"
            kname = "p0_chain_kernel + conv_chain_x3_kernel" if split else "conv_chain_kernel"
            return roof("%s (hbk_embed_clips, %s: %d chained launches per %d-clip chunk)"
                        % (kname, eplan.precision, eplan.n_chains, min(n, 16384)), "mfma",
                        2.0 * eplan.macs_per_clip * n, ms, "TFLOP/s",
                        load_traffic(pmc, ("conv_chain", "p0_chain")),
                        peak=SPLIT_PEAK_TFLOPS if split else FP32_MFMA_PEAK_TFLOPS,
                        peak_basis=("f16 dense MFMA peak / 3 (hi*hi + hi*lo + lo*hi per f32-accurate MAC)"
                                    if split else "f32-input MFMA dense peak"),
                        algorithmic_flops_per_clip=2.0 * eplan.macs_per_clip)
        return roof("augment_kernel (hbk_augment: gain + noise mix + 23040-pt circular FFT reverb, 1 launch)",
                    "hbm", n * AUG_T * 4 * 3, ms, "GB/s", load_traffic(pmc, "augment_kernel"),
                    algorithmic_bytes_per_clip=AUG_T * 4 * 3)

    def cpu_baseline(sample):
        import numpy as np
        from oracle.augment import augment_batch
        from oracle.featurizer import cpu_featurize
        threads = min(16, os.cpu_count() or 1)
        sample = sample or 3000
        x = clips[:sample].cpu().numpy()
        g = default_graph()
        cpu_featurize(x[:4], g, threads=threads)
        c0 = time.perf_counter()
        if augment:
            rng = np.random.default_rng(0)
            nz = rng.standard_normal((sample, AUG_T)).astype(np.float32) * 0.1
            ir = impulse_responses(1, seed=3)[0].numpy()
            x = augment_batch(x[:, :AUG_T], nz, rng.uniform(-10, 15, sample), ir).astype(np.float32)
        cpu_featurize(x, g, threads=threads)
        el = time.perf_counter() - c0
        what = ("augment (numpy fp64 add_noise + rfft reverb) + " if augment else "") + \
            "featurize (reference cost structure: 4x105 mel frames + 16 windows/clip, batch 64; numpy fp32 " \
            "FFT + torch CPU fp32 conv)"
        return {"value": round(sample / el, 2), "unit": "clips/s", "cores": threads, "kind": "port",
                "sample": f"{sample} of the step's clips through oracle/ ({what}), {el:.1f} s"}

    return {
        "step": step, "stages": stages, "roofline": roofline, "cpu_baseline": cpu_baseline,
        "units_per_step": n, "scaling": "weak", "unit": "clips/s",
        "metric": "audio clips/sec featurized+trained, 1.5 s @16 kHz, 1/2/4/8 GPU",
        "data": "synthetic 1.5 s @16 kHz clips (seeded), SE20 stand-in embedding graph"
                + (", synthetic noise bank + IR bank" if augment else ""),
        "config": {"workload": ("configs[2]: 100k clips on-GPU augment (gain + noise mix + IR reverb, p=1"
                                + (", + tanh distortion / colored noise at p=0.25" if args.full_augment else "")
                                + ") -> mel -> embed per GPU") if augment else
                   "configs[1]: 100k clips mel-STFT + speech-embedding forward per GPU",
                   "clips_per_rank": n, "clip_samples": int(clips.shape[1]), "mel_frames_per_clip": N_FRAMES,
                   "windows_per_clip": len(WINDOW_STARTS),
                   "parallelism": f"dp{world} (clip shards, no collective)"},
    }


# --------------------------------------------------------------- config 4 ----
def setup_train(args, dev, rank, world, seed):
    from heybuddy.dataset.training import WakeWordTrainingDatasetIterator
    from heybuddy.trainer import WakeWordTrainer

    g = torch.Generator(device=dev).manual_seed(seed)
    u = torch.randn((16, 96), generator=g, device=dev)
    u /= u.norm()
    pos = torch.randn((100_000, 16, 96), generator=g, device=dev) + 0.5 * u
    adv = torch.randn((100_000, 16, 96), generator=g, device=dev) - 0.25 * u
    neg = torch.randn((200_000, 16, 96), generator=g, device=dev).half()
    gcpu = torch.Generator(device=dev).manual_seed(1234)  # identical batches on every rank
    it = WakeWordTrainingDatasetIterator.default(pos, adv, neg, neg[:100_000], generator=gcpu)
    tr = WakeWordTrainer(checkpoint_dir="/tmp/hb_bench_ck", device=dev)
    batches = iter(it)
    B = it.batch_size
    stream = torch.cuda.current_stream(dev)
    hist = torch.zeros((1 << 16, 8), device=dev)
    counter = [0]

    def step(evs):
        x, y = next(batches)
        if evs:
            evs[0].record(stream)
        tr._step(x, y, 1e-3, 1.0, 1e-4, 0.5, hist, counter[0])
        counter[0] += 1
        if evs:
            evs[1].record(stream)

    P = tr.model.plan.n_params
    flops_per_sample = 2.0 * 559_296  # fwd + bwd MACs/sample (input-layer dX skipped)

    def roofline(name, ms, pmc):
        return roof("hbk_mlp train step (fwd/filter/BCE/bwd + gate/Adam; ~45 launches)", "mfma",
                    flops_per_sample * B / world, ms, "TFLOP/s", None,
                    algorithmic_flops_per_sample=flops_per_sample, params=P, global_batch=B)

    def cpu_baseline(sample):
        import numpy as np
        from oracle import mlp as omlp
        params = omlp.init_params(seed=0)
        rng = np.random.default_rng(0)
        from threadpoolctl import threadpool_limits
        steps = sample or 20
        threads = min(16, os.cpu_count() or 1)
        x = rng.standard_normal((B, 16, 96)).astype(np.float32)
        y = np.concatenate([np.ones(50), np.zeros(B - 50)]).astype(np.int64)
        with threadpool_limits(limits=threads):
            c0 = time.perf_counter()
            for _ in range(steps):
                prob, z, cache = omlp.forward(params, x, dtype=np.float32)
                loss, n, dz = omlp.step_loss_and_dz(prob, y)
                omlp.backward(params, cache, dz, dtype=np.float32)
            el = time.perf_counter() - c0
        return {"value": round(steps * B / el, 1), "unit": "embeddings/s", "cores": threads,
                "kind": "port", "sample": f"{steps} train steps of B={B} through oracle/mlp.py (numpy fp32, "
                                          f"BLAS threads), {el:.1f} s"}

    return {
        "step": step, "stages": ["train_step"], "roofline": roofline, "cpu_baseline": cpu_baseline,
        "units_per_step": B, "scaling": "strong", "unit": "embeddings/s",
        "metric": "wake-word classifier embeddings/sec trained (stage 1, global batch 1100)",
        "data": "synthetic [16,96] embedding pools in HBM (pos N(0,1)+0.5u, adv N(0,1)-0.25u, neg N(0,1) f16)",
        "config": {"workload": "configs[3]: 3-stage classifier training, stage-1 step timing",
                   "global_batch": B, "params": P, "parallelism": f"dp{world} (batch shards + 1 all-reduce/step)"},
    }


if __name__ == "__main__":
    main()
