#!/usr/bin/env python
"""bench.py — the BASELINE.json metric on the MI355X hot path.

Metric: audio clips/sec featurized+trained (1.5 s @ 16 kHz clips), at N GPUs.

Workloads (BASELINE.json configs; --config, default 5 = the headline):
  1  configs[0]: the reference's CPU mel-only case (host oracle, no GPU).
  2  configs[1]: per rank, 100 k clips resident in HBM are featurized exactly
     as SpeechEmbeddings.__call__ does (reference embeddings.py:153-234):
     STFT + 32-bin log-mel (hbk_mel_frames), the speech-embedding graph on the
     16 reference windows per clip (hbk_embed_clips; SE20 stand-in graph — the
     real ONNX graph is absent offline), NaN-row replacement.
  3  configs[2]: the same after on-device augmentation: background-noise mix
     + IR reverb with p forced to 1, one IR per 128-clip batch, and the
     reference's per-batch Gain (p 1.0 by default) (hbk_augment).
  4  configs[3]: classifier training, the reference's 3-stage schedule at
     batch 1,100 / 550 / 275 sampled on the device; embeddings/s trained.
  5  configs[4]: the `heybuddy train` pipeline per rank: placement, the
     reference's augmentation chain at its default probabilities, mel, embed,
     then 1,000 train steps on those clips; clips/s featurized AND trained.
     By default chunk s + 1 is featurized on one stream while chunk s trains
     on another (heybuddy.pipeline, --overlap split:64); the per-stage
     rooflines come from untimed sequential steps.
One step = one pass of the hot path over one batch (100 k clips; for config 4
one 3-stage run).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL). Clips are sharded with no
data-path collective ("weak": every rank featurizes its own 100 k clips);
training runs the reference's batch per rank with one all-reduce of the
gradient bucket per step. The timed region is bracketed by barrier +
synchronize and the max over ranks is reported.

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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=5, choices=(1, 2, 3, 4, 5))
    ap.add_argument("--clips", type=int, default=100_000, help="clips per rank per step (configs 2, 3, 5)")
    ap.add_argument("--cpu-sample", type=int, default=None, help="units timed on the host CPU (~10-30 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--full-augment", action="store_true",
                    help="config 3 plus the reference's tanh distortion and colored noise at their default "
                         "probabilities (0.25 each); not the BASELINE configs[2] workload")
    ap.add_argument("--no-check", action="store_true", help="skip the one-off featurize equality check")
    ap.add_argument("--pitch-prob", type=float, default=0.25,
                    help="config 5: PitchShift probability per batch (the reference's default 0.25)")
    ap.add_argument("--overlap", default=None,
                    help="config 5 (default split:64: 64 CUs train while 192 featurize): "
                         "train chunk s while chunk s + 1 is featurized on a second stream "
                         "(heybuddy.pipeline policies: off, prio, split:N, spill:N; N a multiple of 32, "
                         "i.e. whole CUs of every shader engine of every XCD)")
    ap.add_argument("--train-batch", choices=("per-rank", "global"), default="per-rank",
                    help="config 5 at N > 1: the reference's batch of 1,100 per rank (weak: global batch "
                         "1,100 N, 1,000 steps per rank) or split over the ranks (global batch 1,100, "
                         "N x 1,000 steps per rank)")
    ap.add_argument("--embed-split", type=int, default=-1,
                    help="config 5, pipelined: the embedding's first K fused chains run on the featurize stream, "
                         "the rest (and the NaN replacement) on the train stream after its steps "
                         "(hbk_embed_clips_front / _back; 0: the whole embedding on the featurize stream). "
                         "With the validation + testing passes in the train chunk the train stream carries "
                         "enough: r04g, one box, 0 (no split) 857 k clips/s, partitions featurize 114.5 / "
                         "train 114.1 ms, against 3 / 0.4 776 k (111.1 / 127.2 ms), 3 / 0 785 k. Default (-1, N = 1): "
                         "the graph's chain count with --embed-split-frac 0.2 -- r06, with the train step at 83 us "
                         "the partitions were featurize 109.2 / train 101.5 ms; at 0.2 105.6 / 103.6, headline "
                         "936.5 k against 927.9 k clips/s (two same-box pairs, profiles/r06c_ab_embed_split.log)")
    ap.add_argument("--embed-split-frac", type=float, default=None,
                    help="with --embed-split K: this fraction of each chunk's clips is split after K - 1 "
                         "chains instead (a finer balance of the two streams)")
    ap.add_argument("--validation-steps", type=int, default=250,
                    help="config 5: the reference's validation + testing passes every this many stage steps "
                         "(DEFAULT_VALIDATION_STEPS, trainer.py:496-566; 0 = off): 500 batches of 50 + 1,000 "
                         "validation rows and 500 of 50 + 50 testing rows, dynamic negative weight on the device")
    ap.add_argument("--stage-steps", type=int, default=2,
                    help="overlapped runs: sequential (untimed) steps that time the stages for the rooflines")
    ap.add_argument("--other-configs", default=None,
                    help="with --config 5: these configs (comma list of 1-4) are measured after the headline and "
                         "reported in the same JSON line as configs_other (default 2,3,4,1; '' for none)")
    ap.add_argument("--other-steps", type=int, default=5, help="timed steps of each configs_other measurement")
    ap.add_argument("--other-warmup", type=int, default=2, help="warmup steps of each configs_other measurement")
    ap.add_argument("--pmc", default=None,
                    help="per-kernel HBM bytes per step from rocprofv3 --pmc passes (tools/prof_summary.py JSON; "
                         "default profiles/pmc_c<config>_latest.json)")
    args = ap.parse_args()
    if args.pmc is None:
        args.pmc = os.path.join(ROOT, "profiles", f"pmc_c{args.config}_latest.json")
    if args.other_configs is None:
        args.other_configs = "2,3,4,1"
    if args.overlap is None:  # r03j: split:64 652k clips/s vs split:32 617k with pitch shift on
        args.overlap = "split:64"
    return args


# the split-f16 embedding path's kernels (SE20): streaming chain 0, two-wave chain 1,
# the 16-clip chain 2, the 16-image tail pipeline on the phase-deduplicated tail, the window gather
EMBED_KERNELS = ("p0s_chain_kernel + p1s_chain_kernel + p2s_chain_kernel + t3s_chain_kernel (tail on 2 phase "
                 "images per clip) + embed_gather_kernel")
EMBED_KERNEL_SUBSTR = ("conv_chain", "p0_chain", "p1_chain", "p0s_chain", "p1s_chain", "p2s_chain", "t3s_chain",
                       "embed_gather")
TRAFFIC_SOURCE = [None]
CURRENT_CONFIG = [None]


def load_traffic(path, kernel_substr):
    """HBM bytes per step of the kernels whose name contains kernel_substr (a
    string or a tuple of alternatives), from a tools/prof_summary.py JSON
    ((2 FETCH_SIZE + WRITE_SIZE) KiB per the gfx950 calibration, counted over
    the dispatches of one timed bench step only: between bench.py's profiling
    markers), or None. A summary recorded for another --config (its "config"
    field) is not used: per-step bytes belong to one workload."""
    subs = (kernel_substr,) if isinstance(kernel_substr, str) else tuple(kernel_substr)
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("config") not in (None, CURRENT_CONFIG[0]):
            return None
        kernels = d.get("kernels") or d["regions"]["timed"]["kernels"]
        v = [k for name, k in kernels.items() if any(s in name for s in subs) and "hbm_bytes_per_step" in k]
        if v:
            TRAFFIC_SOURCE[0] = os.path.relpath(path, ROOT)
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
    if traffic is not None:  # PMC bytes are collected in separate rocprofv3 passes, not in this run
        d["traffic_source"] = ("%s (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over one timed step, "
                               "tools/prof_summary.py)" % (TRAFFIC_SOURCE[0],))
    d.update(extra)
    return d


def mel_variant_roofline(x, mplan, n):
    """Untimed, after the measurement: the mel stage with the split-f16 MFMA
    filterbank (hbk_mel_set_variant 1, mel_frames_mfma_kernel) on the same clips,
    beside the default sparse VALU filterbank (north_star names the MFMA form;
    both are reported). HBM algorithmic bytes as the default's entry."""
    from heybuddy.kernels import mel_frames
    mplan.set_variant(1)
    try:
        mel_frames(x, mplan, N_FRAMES)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            mel_frames(x, mplan, N_FRAMES)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
    finally:
        mplan.set_variant(0)
    return roof("mel_frames_mfma_kernel (variant: the 32-mel filterbank as a dense split-f16 "
                "v_mfma_f32_16x16x32_f16 product, 24 MFMAs per 4 frames; %d clips, untimed)" % n, "hbm",
                n * (MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4), ms, "GB/s", None,
                algorithmic_bytes_per_clip=MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4, clips=n)


def prof_mark(tag, dev):
    """hbk_profile_mark_kernel on the current stream, behind a device
    synchronize (outside the timed region): rocprofv3 traces and counter
    passes keep the dispatches between two marks (tools/prof_summary.py)."""
    from heybuddy import _native
    torch.cuda.synchronize(dev)
    _native.check(_native.lib().hbk_profile_mark(tag, _native.stream_ptr(dev)), "hbk_profile_mark")
    torch.cuda.synchronize(dev)


def launch_ranks(args) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment):
    start N ranks under torch.distributed.run as a CHILD process and return
    its exit code. Nothing here touches the GPU (torch is imported, no HIP
    call is made), so the ranks own their devices from the start."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def sub_args(args, config, **over):
    """A copy of the parsed arguments for another measurement in the same run
    (configs_other, the faithful global-batch mode): its own --config, the
    short step counts, its own PMC summary and no profiling markers."""
    a = argparse.Namespace(**vars(args))
    a.config = config
    a.steps, a.warmup = args.other_steps, args.other_warmup
    a.pmc = os.path.join(ROOT, "profiles", f"pmc_c{config}_latest.json")
    a.clips = 100_000
    a.cpu_sample = {2: 1500, 3: 1500, 4: 200}.get(config)
    for k, v in over.items():
        setattr(a, k, v)
    return a


def measure(args, dev, rank, world, marks=True) -> dict:
    """One measurement of --config args.config (2-5) on every rank: setup,
    W warmup steps, then K steps timed between barrier + synchronize on both
    sides; the max over ranks. Returns the JSON line (complete on rank 0)."""
    from heybuddy.synthetic import seed_for
    CURRENT_CONFIG[0] = args.config
    mark = prof_mark if marks else (lambda tag, dev: None)
    setup = {2: setup_featurize, 3: setup_featurize, 4: setup_train, 5: setup_e2e}[args.config]
    job = setup(args, dev, rank, world, seed_for(args.config, rank))

    staged = job.get("staged_step")  # overlapped stages: timed per stage in separate sequential steps
    n_ev = args.stage_steps if staged else args.steps
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(len(job["stages"]) + 1)] for _ in range(n_ev)]
    if staged:  # before the pipelined warmup, which leaves the next chunk's features pending
        staged(None)
        mark(3, dev)
        for k in range(n_ev):
            staged(evs[k])
        torch.cuda.synchronize(dev)
        mark(4, dev)
    for _ in range(args.warmup):
        job["step"](None)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    mark(1, dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        job["step"](None if staged else evs[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mark(2, dev)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    stage_ms = [sum(e[i].elapsed_time(e[i + 1]) for e in evs) / n_ev for i in range(len(job["stages"]))]
    if "rooflines" in job:  # per kernel group (sub-stages timed on their own); the dominant one leads
        roofs = job["rooflines"](dict(zip(job["stages"], stage_ms)), args.pmc)
    else:
        roofs = [job["roofline"](name, ms, args.pmc) for name, ms in zip(job["stages"], stage_ms)]
    # the dominant kernel group by device time (a stage summary that only aggregates
    # groups listed on their own is never the headline entry)
    dom = max(range(len(roofs)), key=lambda i: (not roofs[i].get("summary"), roofs[i]["ms_per_step"]))

    extra = job["extra_rooflines"]() if "extra_rooflines" in job and world == 1 else []
    after = job["after"](elapsed / args.steps * 1e3) if "after" in job else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = job["cpu_baseline"](args.cpu_sample)
    units = job["units_per_step"] * (world if job["scaling"] == "weak" else 1)
    line = {
        "metric": job["metric"], "value": round(units * args.steps / elapsed, 1), "unit": job["unit"],
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": job["scaling"],
        "vs_baseline": None, "dtype": "f32", "data": job["data"], "config": job["config"], "roofline": roofs[dom],
        "roofline_other": [r for i, r in enumerate(roofs) if i != dom] + extra, "cpu_baseline": cpu,
    }
    if after is not None:
        line["cli_path"] = after
    del job, staged, evs  # the next measurement's buffers take their place
    import gc
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return line


def main():
    args = parse()
    CURRENT_CONFIG[0] = args.config
    if args.config == 1:
        print(json.dumps(cpu_mel_only(args)), flush=True)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HBK_BENCH_REHEARSE=1: every rank on cuda:0 over gloo, so that the N > 1
    # code paths (shards, the per-step all-reduce, max-over-ranks timing) run on
    # a one-GPU box; its numbers are not a measurement
    rehearse = os.environ.get("HBK_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    line = measure(args, dev, rank, world)
    if args.config == 5 and world > 1 and args.train_batch == "per-rank":
        # the reference's optimisation on N GPUs: the global batch of 1,100 split over
        # the ranks, N x 1,000 steps per chunk; measured beside the weak-scaling value and named
        g = measure(sub_args(args, 5, train_batch="global"), dev, rank, world, marks=False)
        line["faithful_global_batch"] = {
            k: g[k] for k in ("value", "unit", "steps", "warmup", "ms_per_step", "config", "roofline")}
        line["faithful_global_batch"]["note"] = (
            "the reference's training on N GPUs: global batch 1,100 split over the ranks (SURVEY §8e-2), "
            "N x 1,000 sequential train steps per chunk of N x 100 k clips; `value` above is the weak-scaling "
            "mode (1,100 per rank, 1,000 steps per rank)")
    others = [int(c) for c in args.other_configs.split(",") if c.strip()] if args.config == 5 else []
    if others:
        line["configs_other"] = []
    for c in others:  # BASELINE configs[c - 1] in the same run, after the headline
        if c == 1:
            if rank == 0 and world == 1:
                line["configs_other"].append(cpu_mel_only(sub_args(args, 1)))
            continue
        line["configs_other"].append(measure(sub_args(args, c), dev, rank, world, marks=False))
    if rank == 0:
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
                             tanh_distortion_prob=0.25 if args.full_augment else 0.0,
                             seven_band_prob=0.25 if args.full_augment else 0.0,
                             band_stop_prob=0.25 if args.full_augment else 0.0,
                             pitch_shift_prob=0.25 if args.full_augment else 0.0)  # configs[2]: reverb + noise (+ gain)
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
            kname = (EMBED_KERNELS if split else "conv_chain_kernel")
            return roof("%s (hbk_embed_clips, %s: %d chained launches per %d-clip chunk)"
                        % (kname, eplan.precision, eplan.n_chains, min(n, 16384)), "mfma",
                        2.0 * eplan.macs_per_clip * n, ms, "TFLOP/s",
                        load_traffic(pmc, EMBED_KERNEL_SUBSTR),
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

    def extra_rooflines():
        return [mel_variant_roofline(aug(clips, out=aug_out) if augment else clips, mplan, n)]

    return {
        "step": step, "stages": stages, "roofline": roofline, "cpu_baseline": cpu_baseline,
        "extra_rooflines": extra_rooflines,
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
    """configs[3]: the reference's 3-stage classifier schedule (trainer.py:848-926:
    stage s has 2^s x the steps at 1/2^s the batch and half the lr) on HBM-resident
    embedding pools, through the device-sampled fused train step (train_indexed:
    k1a/k1b/k2/k3/k4 per step on the whole GPU, hipGraph-replayed). A bench step = one pass of
    STEPS_1 stage-1 steps, 2 STEPS_1 stage-2 steps and 4 STEPS_1 stage-3 steps;
    units = embeddings trained (sum of the stages' batches)."""
    import numpy as np
    from heybuddy.trainer import WakeWordTrainer

    g = torch.Generator(device=dev).manual_seed(seed)
    u = torch.randn((16, 96), generator=g, device=dev)
    u /= u.norm()
    pos = torch.randn((100_000, 16, 96), generator=g, device=dev) + 0.5 * u
    adv = torch.randn((100_000, 16, 96), generator=g, device=dev) - 0.25 * u
    pool32 = torch.cat([pos, adv])
    del pos, adv
    neg = torch.randn((200_000, 16, 96), generator=g, device=dev).half()
    tr = WakeWordTrainer(checkpoint_dir="/tmp/hb_bench_ck", device=dev)
    tr.model.train()
    STEPS_1 = 100
    # The reference's stage batches (dataset/training.py:215-231, :436-451): per dataset, positives 50,
    # adversarials 50, large negatives 666 and medium negatives 334 (int(1000 * 2 / 3) and the rest),
    # each multiplied by 0.5 between stages as max(1, int(n * 0.5)): 1,100 -> 550 -> 273 rows. Every rank
    # takes a stride-world share of each dataset's rows (the global batch is split over the ranks; the
    # shares differ by at most one row per dataset). Per stage: 2^s x the steps and the warmup / hold /
    # cosine learning rate of train_epoch (warmup S // 5, hold S // 3, target 1e-3 x 0.5^s; trainer.py:
    # 389-401, :848-926); negative weight 1 (dynamic_negative_weight with no validation set).
    counts = [50, 50, 666, 334]
    stages = []
    global_batches = []
    for s_ in range(3):
        if s_:
            counts = [max(1, int(c * 0.5)) for c in counts]
        global_batches.append(sum(counts))
        P, A, NL, NM = (len(range(rank, c, world)) for c in counts)
        S = STEPS_1 << s_
        gi = torch.Generator(device=dev).manual_seed(seed + 10 + s_)
        rows = torch.cat([torch.randint(0, 100_000, (S, P), generator=gi, device=dev),
                          100_000 + torch.randint(0, 100_000, (S, A), generator=gi, device=dev),
                          -1 - torch.randint(0, 133_000, (S, NL), generator=gi, device=dev),
                          -1 - 133_000 - torch.randint(0, 67_000, (S, NM), generator=gi, device=dev)], 1)
        idx = rows.to(torch.int32).contiguous()
        yv = torch.cat([torch.ones(P), torch.zeros(A + NL + NM)]).to(dev)
        lr = np.asarray(tr.get_learning_rate(np.arange(S), warmup_steps=S // 5, hold_steps=S // 3, total_steps=S,
                                             target_learning_rate=1e-3 * 0.5 ** s_), dtype=np.float32)
        sched = torch.from_numpy(np.stack([lr, np.ones(S, np.float32)], 1)).to(dev)
        stages.append((idx, yv, sched, torch.zeros((S, 8), device=dev)))
    units = sum(int(st[0].shape[0]) * gb for st, gb in zip(stages, global_batches))
    stream = torch.cuda.current_stream(dev)

    def step(evs):
        if evs:
            evs[0].record(stream)
        for idx, yv, sched, hist in stages:
            tr._reset_accumulation()
            tr.train_indexed(idx, yv, sched, pool32=pool32, pool16=neg, history=hist, steps_per_graph=50)
        if evs:
            evs[1].record(stream)

    P_ = tr.model.plan.n_params
    flops_per_sample = 2.0 * 559_296  # fwd + bwd MACs/sample (input-layer dX skipped)
    n_steps = sum(int(st[0].shape[0]) for st in stages)

    def roofline(name, ms, pmc):
        # (the whole GPU: the library's step_v2 picks the v1 kernels there; on a <= 128-CU stream at
        # >= 800 rows it would run k1s / k1c / k3s)
        return roof("k1a/k1b + k2_rows + k3_wgrad + k4_update (fused train step, %d steps over 3 stages)" % n_steps,
                    "latency", flops_per_sample * units / world, ms, "TFLOP/s",
                    load_traffic(pmc, ("k1a_kernel", "k1b_kernel", "k1s_kernel", "k1c_kernel", "k2_rows", "k3_wgrad",
                                       "k3s_kernel", "k4_update")),
                    algorithmic_flops_per_sample=flops_per_sample, params=P_, steps=n_steps,
                    us_per_train_step=round(ms * 1e3 / n_steps, 2))

    def cpu_baseline(sample):
        from oracle import mlp as omlp
        params = omlp.init_params(seed=0)
        rng = np.random.default_rng(0)
        from threadpoolctl import threadpool_limits
        steps = sample or 20
        threads = min(16, os.cpu_count() or 1)
        B1 = 1100
        x = rng.standard_normal((B1, 16, 96)).astype(np.float32)
        y = np.concatenate([np.ones(50), np.zeros(B1 - 50)]).astype(np.int64)
        opt = omlp.Adam(params)
        with threadpool_limits(limits=threads):
            c0 = time.perf_counter()
            for _ in range(steps):
                prob, z, cache = omlp.forward(params, x, dtype=np.float32)
                loss, n, dz = omlp.step_loss_and_dz(prob, y)
                grads = omlp.backward(params, cache, dz, dtype=np.float32)
                params = opt.step(params, grads, 1e-3)
            el = time.perf_counter() - c0
        return {"value": round(steps * B1 / el, 1), "unit": "embeddings/s", "cores": threads,
                "kind": "port", "cpu_model": cpu_model(),
                "sample": f"{steps} stage-1 train steps of B={B1} through oracle/mlp.py incl. Adam (numpy fp32, "
                          f"BLAS threads), {el:.1f} s"}

    def cli_path(ms_indexed):
        """The drop-in's own loop on the same workload: WakeWordTrainer.__call__
        (3 stages of train_epoch, batch sizes halved by the iterator, the stage lr schedule, the final
        checkpoint) over a WakeWordTrainingDatasetIterator of the same device pools, i.e. what `heybuddy
        train` runs; timed after the headline measurement (one warm call, then one timed call) and
        set beside the train_indexed time of the same 700 steps."""
        from heybuddy.dataset.training import WakeWordTrainingDatasetIterator

        views = (pool32[:100_000], pool32[100_000:], neg[:133_000], neg[133_000:])  # one set: the trainer caches
        # the concatenated pools by tensor identity

        def it():
            return WakeWordTrainingDatasetIterator(positive=[(views[0], 50)],
                                                   negative=[(views[1], 50), (views[2], 666), (views[3], 334)],
                                                   device=dev, seed=seed)
        kw = dict(num_steps=STEPS_1, num_stages=3, validation_steps=STEPS_1, checkpoint_steps=10 ** 9,
                  logging_steps=10 ** 9, name="bench_cli")
        tr(it(), **kw)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        c0 = time.perf_counter()
        tr(it(), **kw)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - c0
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item()) * 1e3
        c1 = time.perf_counter()  # the final checkpoint alone (a file write the indexed run does not do)
        tr.save_checkpoint("bench_cli_ckpt_probe")
        ck = (time.perf_counter() - c1) * 1e3
        return {"what": "WakeWordTrainer.__call__ (heybuddy train's loop) over device-pool iterators, 3 stages "
                        "(%d / %d / %d steps at 1,100 / 550 / 273), incl. the final checkpoint" % (
                            STEPS_1, 2 * STEPS_1, 4 * STEPS_1),
                "ms": round(ms, 3), "us_per_train_step": round(ms * 1e3 / n_steps, 2),
                "train_indexed_us_per_train_step": round(ms_indexed * 1e3 / n_steps, 2),
                "ratio_to_train_indexed": round(ms / ms_indexed, 3),
                "checkpoint_ms": round(ck, 3),
                "ratio_to_train_indexed_excl_checkpoint": round((ms - ck) / ms_indexed, 3)}

    return {
        "step": step, "stages": ["train_3stage"], "roofline": roofline, "cpu_baseline": cpu_baseline,
        "after": cli_path,
        "units_per_step": units, "scaling": "strong", "unit": "embeddings/s",
        "metric": "wake-word classifier embeddings/sec trained (3 stages: batch 1100/550/273, steps x1/x2/x4)",
        "data": "synthetic [16,96] embedding pools in HBM (pos N(0,1)+0.5u, adv N(0,1)-0.25u, neg N(0,1) f16), "
                "device-sampled batch indices",
        "config": {"workload": "configs[3]: 3-stage classifier training (%d + %d + %d steps per bench step)"
                               % (STEPS_1, 2 * STEPS_1, 4 * STEPS_1),
                   "stage_batches": global_batches, "lr": "warmup S/5, hold S/3, cosine; 1e-3 x 0.5^stage",
                   "params": P_,
                   "parallelism": f"dp{world} (batch shards + 1 all-reduce/step)"},
    }


# ------------------------------------------------------------ host CPU ----
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def host_threads() -> int:
    """Host cores this process may use (the GPU box's CPU share is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


# --------------------------------------------------------------- config 1 ----
def cpu_mel_only(args):
    """configs[0]: 1,000 synthetic clips, mel spectrogram only, on the host CPU
    (the reference's CPU path: 4 audio windows x 105 frames per clip through
    the mel graph in batches of 64, features.py:203-208). No GPU is touched.
    Reported at all host threads and at 1 thread."""
    import numpy as np
    from oracle.featurizer import cpu_mel_windows
    from heybuddy.synthetic import seed_for, synthetic_clips
    n = args.clips if args.clips != 100_000 else 1000
    clips = synthetic_clips(n, seed=seed_for(1)).numpy()
    threads = host_threads()
    runs = {}
    for th in (threads, 1):
        sub = clips if th == threads else clips[:max(50, n // 10)]
        cpu_mel_windows(sub[:4], threads=th)
        t0 = time.perf_counter()
        out = cpu_mel_windows(sub, threads=th)
        el = time.perf_counter() - t0
        assert out.shape == (sub.shape[0], 420, 32)
        runs[th] = (sub.shape[0] / el, sub.shape[0], el)
    v, nn, el = runs[threads]
    line = {"metric": "audio clips/sec mel-spectrogram (CPU reference path)", "value": round(v, 1),
            "unit": "clips/s", "n_gpus": 0, "steps": 1, "warmup": 1, "ms_per_step": round(el * 1e3, 3),
            "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic 1.5 s @16 kHz clips (seeded)",
            "config": {"workload": "configs[0]: 1,000 synthetic clips, feature_generator mel spectrogram only, "
                                   "CPU reference path (4 x 105 frames per clip, batch 64)",
                       "clips": int(nn), "threads": threads, "cpu_model": cpu_model()},
            "cpu_1thread": {"value": round(runs[1][0], 1), "unit": "clips/s", "cores": 1,
                            "sample": f"{runs[1][1]} clips, {runs[1][2]:.1f} s"}}
    return line


# --------------------------------------------------------------- config 5 ----
def setup_e2e(args, dev, rank, world, seed):
    """configs[4], the headline: the `heybuddy train` pipeline per rank.

    One step = C clips (default 100 k: C/2 TTS-like utterances of the wake
    phrase and C/2 adversarial ones, variable length, resident in HBM) ->
    clip placement (to_target_length) -> the reference's augmentation chain
    at its default probabilities (tanh distortion 0.25 per clip; colored
    noise 0.25, gain 1.0, background noise 0.75, reverb 0.75 per batch of
    128) -> STFT/mel -> speech embedding -> NaN replacement -> the embeddings
    become the positive / adversarial pools of C/100 classifier train steps
    in the reference's stage-1 batch composition (50 positive + 50
    adversarial of THIS step's clips, each used once, + 666 + 334 negatives
    from the precalculated f16 pool), with dropout, filter, BCE, the
    accumulation gate and Adam. Unit = clips featurized AND trained on.
    Data-parallel: every rank runs its own C clips and C/100 steps at the
    reference's batch of 1,100 per rank, with one RCCL all-reduce of the
    gradient bucket per step (weak scaling: the global batch is 1,100 x N)."""
    import numpy as np
    from heybuddy.dataset.augmented import AugmentedAudioGenerator
    from heybuddy.embedding_graph import WINDOW_STARTS
    from heybuddy._native import lib
    from heybuddy.embeddings import default_graph, embed_plan, replace_nan_rows_device
    from heybuddy.kernels import nan_rows_fix
    from heybuddy.kernels import embed_clips, mel_frames
    from heybuddy.spectrogram import default_mel_plan
    from heybuddy.synthetic import impulse_responses, noise_bank, speech_clips
    from heybuddy.trainer import WakeWordTrainer

    n = args.clips
    half = n // 2
    np.random.seed(seed)
    pos, pos_len = speech_clips("hello world", half, seed=seed, device=dev)
    adv, adv_len = speech_clips("hello world", n - half, seed=seed + 1, device=dev, adversarial=True)
    src = torch.cat([pos, adv])
    del pos, adv
    lens = np.concatenate([pos_len, adv_len]).astype(np.int32)
    aug = AugmentedAudioGenerator([], device_id=dev.index, augmentation_dataset=noise_bank(64, seed=seed + 2),
                                  impulse_response_dataset=impulse_responses(32, seed=seed + 3), batch_size=128,
                                  pitch_shift_prob=args.pitch_prob)  # every augmentation at its default
    mplan = default_mel_plan(dev, 32767.0)
    eplan = embed_plan(dev, WINDOW_STARTS)
    pool = torch.empty((n, len(WINDOW_STARTS), 96), dtype=torch.float32, device=dev)
    # embed output before the NaN replacement gathers it into the pool; one extra zero row
    # (the all-NaN case's source: no masked fill over the pool)
    raw_ext = torch.zeros((n + 1,) + tuple(pool.shape[1:]), dtype=torch.float32, device=dev)
    raw = raw_ext[:n]
    # r05: the embedding writes the pool itself and hbk_nan_rows_fix patches its NaN rows in place
    # (no gather copy of the pool, no torch reduction / sort; HBK_NAN_INPLACE=0: the gather form)
    nan_inplace = os.environ.get("HBK_NAN_INPLACE", "1") != "0"
    # pipelined schedule: embedding pools in flight (HBK_PIPE_BUFS, 2 or 3): featurize(c) waits for
    # train(c - nbuf) to release pools[c % nbuf], so a third pool lets the feature stream run a step ahead
    nbuf = max(2, int(os.environ.get("HBK_PIPE_BUFS", "2")))
    nan_ws = [torch.empty(int(lib().hbk_nan_rows_workspace_size(n)), dtype=torch.uint8, device=dev)
              for _ in range(nbuf)]
    nan_seed = [seed * 7919]

    def emb_target(pool_t):
        return pool_t if nan_inplace else raw

    def finish_pool(pool_t, k=0):
        nan_seed[0] += 1
        if nan_inplace:
            nan_rows_fix(pool_t, seed=nan_seed[0], ws=nan_ws[k])
        else:
            replace_nan_rows_device(raw_ext, out=pool_t, zero_row=True)  # no host sync
    # precalculated negatives (the reference's hosted f16 sets): large 2/3, medium 1/3
    g = torch.Generator(device=dev).manual_seed(seed + 4)
    n_neg = 200_000
    neg = torch.randn((n_neg, 16, 96), generator=g, device=dev).half()
    n_large = n_neg * 2 // 3
    P, A, NL, NM = 50, 50, 666, 334
    B = P + A + NL + NM
    S = half // P
    if args.train_batch == "global" and world > 1:
        # the reference's batch of 1,100 is the GLOBAL batch: each rank takes a
        # class-stratified stride-world share of it; all ranks' clips are trained on once on average
        # over world x 1,000 global steps (each rank's positives / adversarials permuted with wrap)
        P, A, NL, NM = (len(range(rank, k, world)) for k in (50, 50, 666, 334))
        B = P + A + NL + NM
        S = (half * world) // 50
    idx = torch.empty((S, B), dtype=torch.int32, device=dev)
    y = torch.cat([torch.ones(P), torch.zeros(B - P)]).to(dev)
    tr = WakeWordTrainer(checkpoint_dir="/tmp/hb_bench_ck", device=dev)
    tr.model.train()  # dropout 0.1 stays on, as in the reference
    steps_total = 5000  # stage-1 LR schedule (warmup 1000, hold 1666, cosine)
    STEP0 = 1000  # a chunk's steps are stage steps STEP0 .. STEP0 + S - 1
    lr = tr.get_learning_rate(np.arange(S) + STEP0, warmup_steps=1000, hold_steps=1666, total_steps=steps_total)
    sched = torch.from_numpy(np.stack([lr, np.ones(S)], 1).astype(np.float32)).to(dev)
    hist = torch.zeros((S, 8), dtype=torch.float32, device=dev)
    # the reference validates (and tests) after every stage step g > 0 with g % validation_steps == 0
    # (trainer.py:496): local steps s of the chunk with (STEP0 + s) % V == 0
    V = args.validation_steps
    val_after = [s_ for s_ in range(S) if V > 0 and (STEP0 + s_) > 0 and (STEP0 + s_) % V == 0]
    ev = None
    if val_after:
        from heybuddy.kernels import place_clips
        from heybuddy.trainer import EvalPasses
        n_eval = 25_000  # DEFAULT_VALIDATION_SAMPLES / DEFAULT_TESTING_*_SAMPLES (constants.py:107-109)

        def featurize_pool(x):
            out = torch.empty((x.shape[0], len(WINDOW_STARTS), 96), dtype=torch.float32, device=dev)
            ext = torch.zeros((x.shape[0] + 1, len(WINDOW_STARTS), 96), dtype=torch.float32, device=dev)
            embed_clips(mel_frames(x, mplan, N_FRAMES), eplan, out=ext[:x.shape[0]])
            replace_nan_rows_device(ext, out=out, zero_row=True)
            return out

        # validation positives: un-augmented, centre-padded wake-phrase clips (get_validation_features,
        # features.py:413-427); validation negatives: the hosted validation set's stand-in (f16)
        vsrc, vlen = speech_clips("hello world", n_eval, seed=seed + 5, device=dev)
        vpre = np.maximum((AUG_T - np.asarray(vlen)) // 2, 0).astype(np.int32)
        vpos = featurize_pool(place_clips(vsrc, np.asarray(vlen, np.int32), vpre, AUG_T))
        del vsrc
        gv = torch.Generator(device=dev).manual_seed(seed + 6)
        vneg = torch.randn((n_eval, 16, 96), generator=gv, device=dev).half()
        # testing: augmented positive / adversarial features (TrainingFeaturesGenerator, testing=True)
        tpos = featurize_pool(aug.augment_device(src[:n_eval], lens[:n_eval]))
        tadv = featurize_pool(aug.augment_device(src[half:half + n_eval], lens[half:half + n_eval]))
        ev = EvalPasses(tr, vpos, vneg, tpos, tadv, seed=seed + 7)
        torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    stages = ["augment", "mel", "embed", "train"]
    neg_pos = [0]

    def sample():
        """Device-side sampler: every featurized clip once (a fresh permutation
        of the step's positives and adversarials), negatives walked through a
        permutation of each pool with wrap-around."""
        k = torch.arange(S * P, device=dev) % half
        idx[:, :P] = torch.randperm(half, device=dev, dtype=torch.int32)[k].view(S, P)
        k = torch.arange(S * A, device=dev) % (n - half)
        idx[:, P:P + A] = half + torch.randperm(n - half, device=dev, dtype=torch.int32)[k].view(S, A)
        o = neg_pos[0]
        k = torch.arange(S * NL, device=dev, dtype=torch.int64)
        idx[:, P + A:P + A + NL] = (-1 - ((o + k) % n_large)).to(torch.int32).view(S, NL)
        k = torch.arange(S * NM, device=dev, dtype=torch.int64)
        idx[:, P + A + NL:] = (-1 - n_large - ((o + k) % (n_neg - n_large))).to(torch.int32).view(S, NM)
        neg_pos[0] = (o + S * NL) % n_large

    eval_events = []  # per staged step: (start, end) events of its evaluation passes
    eval_stream = [None]  # HBK_EVAL_CUS: the evaluation passes' own stream (pipelined schedule only)

    def train_chunk(pool_b, evs=None):
        """The chunk's S stage steps on pool_b, with the evaluation passes after
        the validation steps (all on the current stream, no host sync)."""
        stream_ = torch.cuda.current_stream(dev)
        sample()
        tr._reset_accumulation()
        if not val_after:
            tr.train_indexed(idx, y, sched, pool32=pool_b, pool16=neg, history=hist, steps_per_graph=50)
            return
        # the dynamic negative weight carries over from the previous chunk's last validation
        sched[:, 1].copy_(sched[S - 1:S, 1].expand(S))
        done = 0
        for v_ in val_after:
            tr.train_indexed(idx, y, sched, pool32=pool_b, pool16=neg, history=hist, steps_per_graph=50,
                             n_steps=v_ + 1 - done, continued=done > 0)
            done = v_ + 1
            if evs is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(stream_)
            if eval_stream[0] is not None:
                eval_stream[0].wait_stream(stream_)
                with torch.cuda.stream(eval_stream[0]):
                    ev.run(sched, next_step=done)
                stream_.wait_stream(eval_stream[0])
            else:
                ev.run(sched, next_step=done)
            if evs is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(stream_)
                evs.append((e0, e1))
        if done < S:
            tr.train_indexed(idx, y, sched, pool32=pool_b, pool16=neg, history=hist, steps_per_graph=50,
                             n_steps=S - done, continued=True)

    sub_events = []   # per staged step: (sub-stage, start, end) events of the augment chain
    plan_counts = []  # per staged step: clips each augmentation was applied to

    def step(evs):
        stream = torch.cuda.current_stream(dev)
        prep = aug.prepare_device(src, lens)  # host draws first: the stage events time device work
        if evs:
            ch = prep["chain"]
            plan_counts.append({
                "pitch": sum(int(c.numel()) for _, _, c in ch["pitch"]),
                "eq": 0 if ch["eq"] is None else int(ch["eq"][1].numel()),
                "tanh": 0 if ch["tanh"] is None else int((~torch.isnan(ch["tanh"])).sum()),
                "bandstop": 0 if ch["bandstop"] is None else int(ch["bandstop"][0].numel()),
                "colored": 0 if ch["colored"] is None else int((~torch.isnan(ch["colored"][1])).sum()),
                "mix_reverb": n})
            aug.augmenter.timing = []
            evs[0].record(stream)
        x = aug.augment_device(src, lens, prepared=prep)
        if evs:
            evs[1].record(stream)
            sub_events.append(aug.augmenter.timing)
            aug.augmenter.timing = None
        frames = mel_frames(x, mplan, N_FRAMES)
        if evs:
            evs[2].record(stream)
        embed_clips(frames, eplan, out=emb_target(pool))
        finish_pool(pool)
        if evs:
            evs[3].record(stream)
        eval_events.append([])
        train_chunk(pool, eval_events[-1] if evs else None)
        if evs:
            evs[4].record(stream)

    staged_step = None
    if args.overlap != "off":
        # heybuddy.pipeline: train(s) on the train stream while featurize(s + 1)
        # runs on the feature stream; two embedding pools
        from heybuddy.pipeline import make_streams
        fs, ts, keep = make_streams(dev, args.overlap)
        # the evaluation passes on their own stream, unmasked by default (HBK_EVAL_CUS=N: masked to N
        # CUs; 0: on the train stream), so their workgroups also take the featurize CUs' free slots:
        # 895.2 / 896.4 / 900.4 k against 889.7 / 890.8 / 888.8 k clips/s on the train stream
        # (same box, alternating; profiles/r05l_ab_eval_cus2.log)
        # N > 1: on RCCL too (its count all-reduce is enqueued on the evaluation stream, no host sync);
        # on gloo (tools/rehearse_dp.sh, two ranks sharing cuda:0) the passes stay on the train stream:
        # gloo's all-reduce of the device counts blocks each rank's host until the passes have run, so the
        # extra stream only adds cross-stream waits there -- the records show it slower, not stalled
        # (27.6 against 24.6 s per rehearsal step: gpurun_out/rehearse0.log / rehearse.log)
        eval_default = "-1" if world == 1 or dist.get_backend() == "nccl" else "0"
        n_ecu = int(os.environ.get("HBK_EVAL_CUS", eval_default))
        if n_ecu and world > 1 and dist.get_backend() != "nccl":
            raise SystemExit("HBK_EVAL_CUS != 0 with %d gloo ranks: the evaluation passes' own stream needs a "
                             "collective enqueued on it (RCCL); gloo's host-blocking count all-reduce would "
                             "serialise it against the train stream (DESIGN.md §6)" % world)
        if n_ecu < 0:
            n_ecu = torch.cuda.get_device_properties(dev).multi_processor_count
        if n_ecu and ev is not None:
            from heybuddy.pipeline import masked_stream, train_cu_set
            n_all = torch.cuda.get_device_properties(dev).multi_processor_count
            if n_ecu >= n_all:
                eval_stream[0] = torch.cuda.Stream(dev)
            else:
                es = masked_stream(dev, train_cu_set(n_all, n_ecu))
                keep.append(es)
                eval_stream[0] = es.stream
        pools = [pool] + [torch.empty_like(pool) for _ in range(nbuf - 1)]
        feat_done = [torch.cuda.Event() for _ in range(nbuf)]
        train_done = [torch.cuda.Event() for _ in range(nbuf)]
        count = [0]
        staged_step = step

        host_log = os.environ.get("HBK_BENCH_HOSTTIME")
        # HBK_BENCH_PARTITION=1: each partition's device time per step (events on
        # its own stream, from its first kernel to its last), printed at exit
        part = [] if os.environ.get("HBK_BENCH_PARTITION") else None
        if part is not None:
            import atexit

            def _report():
                torch.cuda.synchronize(dev)
                for name in ("featurize", "train"):
                    ms = [a.elapsed_time(b) for k, a, b in part if k == name][2:]  # past the warmup
                    if ms:
                        print("partition %s: %.2f ms per step (%d steps)" % (name, sum(ms) / len(ms), len(ms)),
                              file=sys.stderr, flush=True)
            atexit.register(_report)

        def mark(name, stream):
            if part is None:
                return None
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            return e

        # --embed-split K: the partitions are unbalanced (featurize ~127 ms on 192 CUs,
        # train ~93 ms on 64 at split:64), so the embedding's last chains of chunk c + 1
        # run on the train stream after train(c): its front half writes mid[b] on the
        # feature stream, its back half reads it on the train stream
        # (K = n_chains: only the --embed-split-frac clips are split, after K - 1 chains)
        if args.embed_split < 0:  # default: a fifth of the clips' last chains on the train stream at N = 1
            args.embed_split = eplan.n_chains
            if args.embed_split_frac is None:
                # N > 1: none -- the train stream then also folds the weight-gradient slabs and all-reduces
                # the bucket every step (r06_dp_probe.log: +9 us per step before the collective itself), so
                # the train partition is the longer one and the embedding stays on the featurize stream
                args.embed_split_frac = 0.2 if world == 1 else 0.0
        if args.embed_split_frac is None:
            args.embed_split_frac = 0.0
        K = args.embed_split if 0 < args.embed_split <= eplan.n_chains else 0
        whole = K == eplan.n_chains  # the rest of the clips: the whole embedding on the featurize stream
        # --embed-split-frac f: clips [0, a1) split after K - 1 chains, the rest after K
        a1 = int(round(n * args.embed_split_frac)) if K > 1 else 0
        a1 = min(max(a1, 0), n)
        mids = [torch.empty((n - a1, eplan.mid_floats(K)), dtype=torch.float32, device=dev)
                for _ in range(nbuf)] if K and not whole else []
        mids1 = [torch.empty((a1, eplan.mid_floats(K - 1)), dtype=torch.float32, device=dev)
                 for _ in range(nbuf)] if a1 else []
        front_done = [torch.cuda.Event() for _ in range(nbuf)]

        def featurize(c):
            b = c % nbuf
            with torch.cuda.stream(fs):
                fs.wait_event(train_done[b])  # train(c - nbuf) has finished reading pools[b] (and back(c - nbuf) mids[b])
                e0 = mark("featurize", fs)
                x = aug.augment_device(src, lens)
                frames = mel_frames(x, mplan, N_FRAMES)
                if K:
                    if a1:
                        eplan.clips_front(frames[:a1], K - 1, mids1[b])
                    if a1 < n and whole:
                        embed_clips(frames[a1:], eplan, out=emb_target(pools[b])[a1:])
                    elif a1 < n:
                        eplan.clips_front(frames[a1:], K, mids[b])
                    front_done[b].record(fs)
                else:
                    embed_clips(frames, eplan, out=emb_target(pools[b]))
                    finish_pool(pools[b], b)
                    feat_done[b].record(fs)
                if part is not None:
                    part.append(("featurize", e0, mark("featurize", fs)))

        def featurize_back(c):
            """Chunk c's embedding back half + NaN replacement on the train stream."""
            b = c % nbuf
            with torch.cuda.stream(ts):
                ts.wait_event(front_done[b])
                if a1:
                    eplan.clips_back(mids1[b], a1, K - 1, emb_target(pools[b])[:a1])
                if a1 < n and not whole:
                    eplan.clips_back(mids[b], n - a1, K, emb_target(pools[b])[a1:])
                finish_pool(pools[b], b)
                feat_done[b].record(ts)

        def step(evs):  # noqa: F811
            # chunk c+1 is featurized while chunk c trains; its work is queued
            # FIRST: 1,000 train steps are ~5,000 packets, and a full hardware
            # queue blocks the host until the device drains it
            c = count[0]
            count[0] += 1
            if c == 0:
                featurize(0)  # pipeline fill (first warmup step)
                if K:
                    featurize_back(0)
            h0 = time.perf_counter()
            featurize(c + 1)
            h1 = time.perf_counter()
            b = c % nbuf
            with torch.cuda.stream(ts):
                ts.wait_event(feat_done[b])
                e0 = mark("train", ts)
                train_chunk(pools[b])
                train_done[b].record(ts)
            if K:
                featurize_back(c + 1)
            if part is not None:
                part.append(("train", e0, mark("train", ts)))
            if host_log:
                print("host ms: featurize enqueue %.1f, train enqueue %.1f" % (
                    1e3 * (h1 - h0), 1e3 * (time.perf_counter() - h1)), file=sys.stderr, flush=True)
        step.keep = keep  # the CU-masked streams live as long as the step

    flops_step = 2.0 * 559_296 * B
    _fft = 2.5 * 250 * np.log2(250)
    PITCH_FLOP_PER_CLIP = 3292 * _fft + 3372 * 126 * 16 + 3372 * (_fft + 250) + 23044 * 2 * 142

    def rooflines(stage_ms, pmc):
        """Per kernel group, each against its own bound: the augment chain's
        sub-stages (timed by their own events on the stream they run on), mel,
        embed and the train step; the whole augment stage is kept as a summary
        entry. Algorithmic work per unit is stated in each entry."""
        torch.cuda.synchronize(dev)
        sub_ms, cnt = {}, {}
        for evl, pc in zip(sub_events, plan_counts):
            for name, a, b in evl:
                sub_ms[name] = sub_ms.get(name, 0.0) + a.elapsed_time(b) / len(sub_events)
            for k_, v_ in pc.items():
                cnt[k_] = cnt.get(k_, 0) + v_ / len(plan_counts)
        out = []
        if sub_ms.get("pitch"):
            m = cnt["pitch"]
            out.append(roof("ps_vocoder_kernel + ps_resample_mfma_kernel (hbk_pitch_shift: %.0f clips shifted per step, "
                            "p = %g per batch of 128)" % (m, args.pitch_prob), "valu", PITCH_FLOP_PER_CLIP * m,
                            sub_ms["pitch"], "TFLOP/s", load_traffic(pmc, ("ps_vocoder", "ps_resample", "ps_taps")),
                            peak=157.3, peak_basis="f32 vector peak (MI355X_MICROARCH.md)",
                            algorithmic_flops_per_clip=round(PITCH_FLOP_PER_CLIP),
                            flops_basis="FFT-based count of the reference's algorithm per shifted clip: stft 3,292 x "
                                        "2.5 N log2 N (N = 250) + vocoder 3,372 x 126 x 16 + istft 3,372 x (2.5 N log2 N "
                                        "+ 250) + resample 23,044 x 2 x 142", clips=round(m)))
        per_clip = {"mix_reverb": (AUG_T * 4 * 3, "augment_kernel (colored-noise mix of the batches that drew it, folded "
                                   "into its prologue (+ colored_group_kernel: one coloured second per such batch) + gain + "
                                   "noise mix + 23040-pt FFT reverb, every clip)",
                                   ("augment_kernel", "colored_group", "colored_noise"),
                                   "x + noise read, y written (the coloured seconds are L2-resident, 64 KB per batch)"),
                    "eq": (AUG_T * 4 * 2, "eq_kernel (7-band EQ, the clips whose coin came up)", ("eq_kernel",),
                           "x read + y written"),
                    "tanh": (AUG_T * 4 * 2, "tanh_distortion_kernel (the clips whose coin came up)",
                             ("tanh_distortion",), "x read + y written"),
                    "bandstop": (AUG_T * 4 * 2, "band_stop_kernel (+ sums / spectrum, the batches whose coin came up)",
                                 ("band_stop",), "x read + y written"),
                    "colored": (AUG_T * 4 * 2, "colored_group_kernel + colored_mix_kernel (+ colored_noise_kernel for "
                                "clips outside a group; the batches whose coin came up)",
                                ("colored_noise", "colored_mix", "colored_group"), "x read + y written")}
        for name, (bpc, kname, subs, basis) in per_clip.items():
            if sub_ms.get(name):
                m = cnt.get(name, n)
                out.append(roof(kname, "hbm", bpc * m, sub_ms[name], "GB/s", load_traffic(pmc, subs),
                                algorithmic_bytes_per_clip=bpc, bytes_basis=basis, clips=round(m)))
        ev_ms = 0.0
        staged_ev = [e for e in eval_events if e]
        if staged_ev:
            ev_ms = sum(a.elapsed_time(b) for evl in staged_ev for a, b in evl) / len(staged_ev)
            rows = ev.rows_per_pass * len(val_after)
            out.append(roof("kv_gemm_kernel (input GEMM + the rest of the network, one launch per pool; + kv_prep / "
                            "kv_finish): the validation and "
                            "testing passes, %d per chunk of %d rows each (dropout on)" % (len(val_after),
                                                                                           ev.rows_per_pass),
                            "mfma", 2.0 * 251_968 * rows, ev_ms, "TFLOP/s",
                            load_traffic(pmc, ("kv_gemm", "kv_prep", "kv_finish")), peak=SPLIT_PEAK_TFLOPS,
                            peak_basis="f16 dense MFMA peak / 3 (split-f16 products; f16 pool rows need 2)",
                            algorithmic_flops_per_row=2.0 * 251_968, rows=rows))
        for name in ("augment", "mel", "embed", "train"):
            out.append(roofline(name, stage_ms[name] - (ev_ms if name == "train" else 0.0), pmc))
        return out

    def roofline(name, ms, pmc):
        if name == "augment":
            return roof("augment stage (summary; its kernels are listed on their own): place_kernel + eq_kernel + tanh_distortion_kernel + ps_*_kernel + band_stop_kernel + "
                        "colored_noise_kernel + augment_kernel (placement, 7-band EQ, tanh, pitch shift, band-stop, "
                        "colored noise, gain + noise mix + 23040-pt FFT reverb)", "hbm",
                        n * AUG_T * 4 * 2, ms, "GB/s", load_traffic(pmc, ("place_kernel", "augment_kernel", "eq_kernel",
                                                                          "band_stop", "colored_", "ps_",
                                                                          "tanh_distortion")),
                        algorithmic_bytes_per_clip=AUG_T * 4 * 2, summary=True,
                        bytes_basis="placed clip written + augmented clip written in place (92,160 B each); "
                                    "the chain's re-reads of the in-place buffer are not counted")
        if name == "mel":
            return roof("mel_frames_v2_kernel (hbk_mel_frames)", "hbm",
                        n * (MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4), ms, "GB/s", load_traffic(pmc, "mel_frames"),
                        algorithmic_bytes_per_clip=MEL_READ_SAMPLES * 4 + N_FRAMES * 32 * 4)
        if name == "embed":
            split = eplan.precision == "split"
            return roof("%s (hbk_embed_clips)" % EMBED_KERNELS, "mfma",
                        2.0 * eplan.macs_per_clip * n, ms, "TFLOP/s",
                        load_traffic(pmc, EMBED_KERNEL_SUBSTR),
                        peak=SPLIT_PEAK_TFLOPS if split else FP32_MFMA_PEAK_TFLOPS,
                        peak_basis="f16 dense MFMA peak / 3 (hi*hi + hi*lo + lo*hi per f32-accurate MAC)",
                        algorithmic_flops_per_clip=2.0 * eplan.macs_per_clip)
        # (the stage region runs on the whole GPU, where the library's step_v2 picks v1; the
        # pipelined headline's 64-CU train partition runs v2 at B = 1,100)
        step_kernels = "k1a + k1b + k2_rows + k3_wgrad + k4_update"
        return roof("%s (fused train step, %d steps of B=%d)" % (step_kernels, S, B),
                    "latency", flops_step * S, ms, "TFLOP/s",
                    load_traffic(pmc, ("k1a_kernel", "k1s_kernel", "k1b_kernel", "k1c_kernel", "k2_rows", "k3_wgrad",
                                       "k3s_kernel", "k4_update")),
                    algorithmic_flops_per_sample=2.0 * 559_296, steps=S, batch=B,
                    us_per_train_step=round(ms * 1e3 / S, 2),
                    bound_note="a chain of dependent small GEMMs at B = 1,100 (PMC: MFMA busy a few %): latency-"
                               "bound; frac is against the f32 MFMA peak (157.3 TF/s)")

    def cpu_baseline(sample_n):
        """The same pipeline on the host CPU (oracle/): placement, the
        reference's whole augmentation chain (oracle.augment.augment_chain:
        7-band EQ and tanh per clip; pitch shift, band-stop, colored noise,
        gain, background noise and reverb per batch of 128, at the default
        probabilities, each per-batch coin stratified so that the sample holds
        round(p * batches) of each), featurize at the reference's cost
        structure, then the train steps of exactly those clips (50 positives +
        50 adversarials of the sample per step + 1,000 negatives, numpy fp32
        forward / backward / Adam at B = 1,100). Featurization runs on a pool
        of single-threaded worker processes, one 128-clip batch per job
        (oracle.pipeline_cpu; the reference's feature generation also runs in
        worker processes); the 1-thread figure is the same work timed as the
        workers' summed busy time plus the train steps on one BLAS thread."""
        from oracle.pipeline_cpu import featurize_pool
        from oracle import mlp as omlp
        from threadpoolctl import threadpool_limits
        gr = default_graph()
        nb_cpu = [v.numpy() for v in noise_bank(64, seed=seed + 2)]
        ir_cpu = [v.numpy() for v in impulse_responses(32, seed=seed + 3)]
        th = host_threads()
        m = sample_n or 1024  # 8 batches of 128 (32 jobs of 32 clips): ~40 s of single-thread work
        # half positives, half adversarials, as the step's clips
        rows = np.concatenate([np.arange(m // 2), half + np.arange(m - m // 2)])
        order = np.random.default_rng(0).permutation(m)  # batches mix both halves, as the device sampler's
        rows = rows[order]
        xs, ls = src[rows].cpu().numpy(), lens[rows]
        emb, wall, busy, counts = featurize_pool(xs, ls, nb_cpu, ir_cpu, gr, th, seed=seed)
        emb = emb[np.argsort(order)]  # back to [positives | adversarials]
        steps = max(1, (m // 2) // P)
        eval_rows = int(round(ev.rows_per_pass * steps / V)) if ev is not None else 0
        yy = np.concatenate([np.ones(P), np.zeros(B - P)]).astype(np.int64)
        train_s = {}
        for tth in (th, 1):
            rng = np.random.default_rng(1)
            with threadpool_limits(limits=tth):
                torch.set_num_threads(tth)
                params = omlp.init_params(seed=0)
                opt = omlp.Adam(params)
                t0 = time.perf_counter()
                for s_ in range(steps):
                    pos_ = emb[s_ * P:(s_ + 1) * P]
                    adv_ = emb[m // 2 + s_ * A:m // 2 + (s_ + 1) * A]
                    negs = rng.standard_normal((B - P - A, 16, 96)).astype(np.float16).astype(np.float32)
                    xb = np.concatenate([pos_, adv_, negs]).astype(np.float32)
                    prob, z, cache = omlp.forward(params, xb, dtype=np.float32)
                    loss, nsel, dz = omlp.step_loss_and_dz(prob, yy)
                    grads = omlp.backward(params, cache, dz, dtype=np.float32)
                    params = opt.step(params, grads, 1e-3)
                # the evaluation passes' share of these steps: rows_per_pass x steps / validation_steps
                # forward rows (dropout on, the reference's validation loop without .eval())
                for r0_ in range(0, eval_rows, 4096):
                    xr = rng.standard_normal((min(4096, eval_rows - r0_), 16, 96)).astype(np.float32)
                    xr *= (rng.random(xr.shape) >= 0.1) / np.float32(0.9)
                    omlp.forward(params, xr, dtype=np.float32)
                train_s[tth] = time.perf_counter() - t0
        torch.set_num_threads(th)
        el, el1 = wall + train_s[th], busy + train_s[1]
        return {"value": round(m / el, 2), "unit": "clips/s", "cores": th, "kind": "port",
                "cpu_model": cpu_model(),
                "sample": f"{m} of the step's clips through oracle/ on {th} single-threaded worker processes "
                          f"(jobs of 32 clips of a 128-clip batch, oracle/pipeline_cpu.py): placement + the full augmentation "
                          f"chain (7-band EQ, tanh, pitch shift [float32 torch.stft/istft + phase vocoder + sinc "
                          f"resample], band-stop, colored noise, gain, background noise, reverb; applied: "
                          f"{counts}) + featurize at the reference's cost structure (4 x 105 mel frames, "
                          f"16 windows per clip, batch 64) in {wall:.1f} s wall, then {steps} train steps of B={B} "
                          f"on those clips' embeddings incl. Adam and the evaluation passes' share ({eval_rows} "
                          f"forward rows) ({th} BLAS threads) in {train_s[th]:.1f} s",
                "value_1thread": round(m / el1, 2),
                "sample_1thread": f"the same {m} clips and {steps} train steps on one thread: featurize = the "
                                  f"workers' summed busy time {busy:.1f} s, train {train_s[1]:.1f} s",
                "speedup_vs_1thread": round(el1 / el, 2)}

    def extra_rooflines():
        """Untimed, after the measurement: the embedding on the generic
        split-f16 chain kernel alone (HBK_EMBED_NO_P0 / NO_P1: what a graph
        without SE20's chain shapes would run), on one 16,384-clip chunk."""
        from heybuddy.kernels import EmbedPlan
        m = min(n, 16384)
        frames = mel_frames(aug.augment_device(src[:m], lens[:m]), mplan, N_FRAMES)
        saved = {k: os.environ.get(k) for k in ("HBK_EMBED_NO_P0", "HBK_EMBED_NO_P1", "HBK_EMBED_NO_P2S",
                                                "HBK_EMBED_NO_T3S")}
        os.environ.update({"HBK_EMBED_NO_P0": "1", "HBK_EMBED_NO_P1": "1", "HBK_EMBED_NO_P2S": "1",
                           "HBK_EMBED_NO_T3S": "1"})
        try:
            gplan = EmbedPlan(default_graph(), starts=WINDOW_STARTS, device=dev, precision=eplan.precision)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        out = torch.empty((m, len(WINDOW_STARTS), 96), dtype=torch.float32, device=dev)
        embed_clips(frames, gplan, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            embed_clips(frames, gplan, out=out)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / 3
        extra = [roof("conv_chain_x3_kernel only (HBK_EMBED_NO_P0 / P1 / P2S / T3S: the generic split-f16 chain "
                      "kernel on every chain, as for a graph without SE20's chain shapes; %d clips, untimed)" % m,
                      "mfma", 2.0 * gplan.macs_per_clip * m, ms, "TFLOP/s", None, peak=SPLIT_PEAK_TFLOPS,
                      peak_basis="f16 dense MFMA peak / 3", clips=m)]
        extra.append(mel_variant_roofline(aug.augment_device(src, lens), mplan, n))
        return extra

    return {
        "step": step, "staged_step": staged_step, "stages": stages, "roofline": roofline, "rooflines": rooflines,
        "extra_rooflines": extra_rooflines,
        "cpu_baseline": cpu_baseline, "units_per_step": n, "scaling": "weak", "unit": "clips/s",
        "metric": "audio clips/sec featurized+trained, 1.5 s @16 kHz, 1/2/4/8 GPU",
        "data": "synthetic TTS-like utterances (seeded, 0.3-1.5 s), synthetic noise + IR banks, synthetic "
                "f16 negative pool; SE20 stand-in embedding graph",
        "config": {"workload": "configs[4]: end-to-end heybuddy-train pipeline per GPU: placement -> augment "
                               "(reference default probabilities: 7-band EQ, tanh, pitch shift p=%g, band-stop, colored "
                               "noise, gain, background noise, reverb) -> mel -> embed -> %d train steps (B=%d: 50 pos "
                               "+ 50 adv of the step's clips + 1000 f16 negatives)" % (args.pitch_prob, S, B),
                   "clips_per_rank": n, "train_steps_per_rank": S, "train_batch_per_rank": B,
                   "train_batch_mode": ("global: the reference's 1,100 split over the ranks" if
                                        args.train_batch == "global" and world > 1 else
                                        "per-rank: 1,100 per rank (global batch 1,100 x N)"),
                   "negative_pool": f"{n_neg} x [16,96] f16",
                   "validation": ("off" if not val_after else
                                  f"every {V} stage steps (stage steps {STEP0}..{STEP0 + S - 1}: after local steps "
                                  f"{val_after}): validation = 500 batches of 50 positives (25,000 un-augmented "
                                  f"features) + 1,000 negatives (25,000 f16), testing = 500 batches of 50 positives "
                                  f"+ 50 adversarial (25,000 each, augmented); dropout on; counts, false positives "
                                  f"per hour and the dynamic negative weight (x2 above 1.5 / h, /2 floor 1) on the "
                                  f"device; {ev.rows_per_pass} rows per pass"),
                   "parallelism": f"dp{world} (clip shards; 1 all-reduce of the 1,025,700-B bucket per train step)",
                   "schedule": ("sequential: featurize(s) then train(s)" if args.overlap == "off" else
                                f"pipelined (heybuddy.pipeline {args.overlap}): featurize(s + 1) on one stream while "
                                f"train(s) runs on another"
                                + (f", then the embedding's chains >= {args.embed_split} of chunk s + 1 on the train "
                                   "stream (hbk_embed_clips_back)" if 0 < args.embed_split < eplan.n_chains else "")
                                + (f" (chains >= {args.embed_split - 1} for {args.embed_split_frac:.0%} of the clips)"
                                   if 1 < args.embed_split < eplan.n_chains and args.embed_split_frac > 0 else "")
                                + (f", then the embedding's chains >= {args.embed_split - 1} of {args.embed_split_frac:.0%}"
                                   " of chunk s + 1's clips on the train stream (hbk_embed_clips_back)"
                                   if args.embed_split == eplan.n_chains and args.embed_split_frac > 0 else "")
                                + (", the evaluation passes on a stream of their own over "
                                   + ("all CUs" if eval_stream[0] is not None and not isinstance(
                                       eval_stream[0], torch.cuda.ExternalStream) else "a CU-masked set")
                                   if eval_stream[0] is not None else "")
                                + f"; per-stage ms from {args.stage_steps} sequential steps")},
    }


if __name__ == "__main__":
    main()
