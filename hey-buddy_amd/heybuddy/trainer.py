"""Drop-in for heybuddy.trainer (reference src/python/heybuddy/trainer.py).

``WakeWordTrainer`` keeps the reference's constructor, ``get_learning_rate``,
``loss``, ``num_false_positives``, ``train_epoch`` (same arguments, same
11-tuple of histories) and the 3-stage ``__call__``, checkpoints
(``{name}.pt`` + ``{name}_optimizer.pt``) and ``resume``. Each optimisation
step is the fused HIP train step of libhbk.so:

  hbk_mlp_train_fwd_bwd  forward (+ input dropout), high-loss filter, weighted
                         BCE, backward -> gradient bucket + statistics
  all_reduce(bucket)     RCCL, only when torch.distributed is initialised
                         (captured into the step's hipGraph on RCCL):
                         every rank trains on a 1/world slice of each batch
  hbk_mlp_gate_adam      the reference's < 128-sample accumulation gate on the
                         global statistics, then Adam iff it fires

No host synchronisation per step (the reference forces gc.collect(),
empty_cache() and synchronize() every step, trainer.py:592-594); the loss /
recall / false-positive histories are rebuilt from a device-side per-step
record with the reference's bookkeeping rules (trainer.py:443-494).
"""
from __future__ import annotations

import contextlib
import math
import os
import random
from time import perf_counter
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from heybuddy.constants import *  # noqa: F401,F403
from heybuddy.constants import (DEFAULT_ACTIVATION_THRESHOLD, DEFAULT_ARCHITECTURE,
                                DEFAULT_BATCH_SIZE_ADJUST_RATIO, DEFAULT_CHECKPOINT_STEPS,
                                DEFAULT_DYNAMIC_NEGATIVE_WEIGHT, DEFAULT_HEADS,
                                DEFAULT_HIGH_LOSS_THRESHOLD, DEFAULT_HOLD_STEPS, DEFAULT_LAYER_DIM,
                                DEFAULT_LAYERS, DEFAULT_LEARNING_RATE,
                                DEFAULT_LEARNING_RATE_ADJUST_RATIO, DEFAULT_LOGGING_STEPS,
                                DEFAULT_NEGATIVE_WEIGHT, DEFAULT_NEGATIVE_WEIGHT_ADJUST_RATIO,
                                DEFAULT_STAGES, DEFAULT_STEP_ADJUST_RATIO, DEFAULT_STEPS,
                                DEFAULT_TARGET_FALSE_POSITIVE_RATE, DEFAULT_VALIDATION_STEPS,
                                DEFAULT_WARMUP_STEPS)
from heybuddy import distributed
from heybuddy.pipeline import capture_stream
from heybuddy.util import logger
from heybuddy.wakeword import WakeWordMLPModel

__all__ = ["Trainer", "WakeWordTrainer", "EvalPasses"]

BETAS = (0.9, 0.999)
EPS = 1e-8


class Trainer(nn.Module):
    """Base trainer: checkpoint dir, model, optimizer, LR schedule (trainer.py:27-204)."""

    def __init__(self, checkpoint_dir: str = "./checkpoints", learning_rate: float = DEFAULT_LEARNING_RATE,
                 device: Optional[Union[str, torch.device]] = None, **model_kwargs: Any) -> None:
        super().__init__()
        self.checkpoint_dir = os.path.abspath(checkpoint_dir)
        os.makedirs(self.checkpoint_dir, exist_ok=True)
        self.model = self.create_model(**model_kwargs)
        if device is None and torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
        if device is not None:
            self.model.to(device)
        self.learning_rate = learning_rate
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=learning_rate)
        self._init_state()
        self._weights_synced = False

    def sync_initial_weights(self, group: Optional["dist.ProcessGroup"] = None) -> None:
        """Data-parallel: overwrite this rank's parameters with rank 0's, so that
        every rank starts from the same weights (the identical all-reduced Adam
        updates then keep them identical). A collective over ``group``: the
        first data-parallel train call (train_epoch's steps, train_indexed)
        runs it; constructing a trainer is rank-local (a rank-0-only export or
        evaluation tool builds one without a partner)."""
        with torch.no_grad():
            distributed.broadcast_(self.model.flat_parameters, group=group)
        self._weights_synced = True

    def _ensure_synced(self) -> None:
        if not self._weights_synced and distributed.reduces():
            self.sync_initial_weights()

    def create_model(self, **kwargs: Any) -> nn.Module:
        raise NotImplementedError()

    # device-resident optimiser state (the kernels' flat layout)
    def _init_state(self) -> None:
        flat = self.model.flat_parameters
        dev = flat.device
        self._m = torch.zeros_like(flat)
        self._v = torch.zeros_like(flat)
        # generic path (hbk_mlp_gate_adam): [acc_samples, acc_steps, adam t, step]
        self._state = torch.tensor([0.0, 1.0, 0.0, 0.0], dtype=torch.float32, device=dev)
        self._ctrl = torch.zeros(4, dtype=torch.float32, device=dev)
        # fused path (hbk_mlp_step_*): ping-ponged [2][8] state, `_parity` = half of the next step
        self._fstate = torch.tensor([0.0, 1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0] * 2, dtype=torch.float32, device=dev)
        self._parity = 0
        self._bucket = torch.zeros(flat.numel() + self.model.plan.N_STATS, dtype=torch.float32, device=dev)
        self._graphs = {}

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        if hasattr(self, "_m"):
            self._m, self._v = fn(self._m), fn(self._v)
            self._state, self._ctrl, self._bucket = fn(self._state), fn(self._ctrl), fn(self._bucket)
            self._fstate = fn(self._fstate)
            self._graphs = {}
        return self

    @property
    def device(self) -> torch.device:
        return self.model.device

    @property
    def _fused(self) -> bool:
        return self.model.plan.fused and self.device.type == "cuda"

    def _adam_t(self) -> float:
        if self._fused:
            return float(self._fstate[8 * self._parity + 2].item())
        return float(self._state[2].item())

    def _reset_accumulation(self, salt: int = 0) -> None:
        """Start of an epoch (trainer.py:377-378): accumulated samples 0,
        accumulation steps 1, step index 0; the Adam step count is kept.
        Device-side only (no host sync)."""
        st = self._fstate.view(2, 8)
        st[1 - self._parity].copy_(st[self._parity])
        st[:, 0] = 0.0
        st[:, 1] = 1.0
        st[:, 3] = 0.0
        st[:, 4] = float(salt % (1 << 24))
        self._parity = 0
        self._state[0] = 0.0
        self._state[1] = 1.0
        self._state[3] = 0.0

    def get_learning_rate(self, step: int, warmup_steps: int = 0, hold_steps: int = 0, total_steps: int = 0,
                          start_learning_rate: float = 0.0,
                          target_learning_rate: float = DEFAULT_LEARNING_RATE) -> np.ndarray:
        """Cosine decay with linear warmup and a hold (trainer.py:127-156)."""
        learning_rate = 0.5 * target_learning_rate * (1 + np.cos(
            np.pi * (step - warmup_steps - hold_steps) / float(total_steps - warmup_steps - hold_steps)))
        warmup_learning_rate = target_learning_rate * (step / warmup_steps) if warmup_steps > 0 else 0.0
        if hold_steps > 0:
            learning_rate = np.where(step > warmup_steps + hold_steps, learning_rate, target_learning_rate)
        return np.where(step < warmup_steps, warmup_learning_rate, learning_rate)

    # -- checkpoints (trainer.py:186-198, resume :54-118) ----------------------
    def _sync_torch_optimizer(self) -> None:
        """Expose the kernels' Adam state through torch.optim.Adam's state_dict."""
        t = int(self._adam_t())
        views_m = self.model.plan.views(self._m)
        views_v = self.model.plan.views(self._v)
        for name, p in self.model.named_parameters():
            st = self.optimizer.state[p]
            st["step"] = torch.tensor(float(t))
            st["exp_avg"] = views_m[name]
            st["exp_avg_sq"] = views_v[name]

    def save_checkpoint(self, name: str, optimizer: bool = True) -> None:
        torch.save(self.model.state_dict(), os.path.join(self.checkpoint_dir, f"{name}.pt"))
        if optimizer:
            self._sync_torch_optimizer()
            torch.save(self.optimizer.state_dict(), os.path.join(self.checkpoint_dir, f"{name}_optimizer.pt"))

    def resume(self, name: str) -> None:
        files = os.listdir(self.checkpoint_dir)
        models = sorted(((f, os.path.getmtime(os.path.join(self.checkpoint_dir, f))) for f in files
                         if f.startswith(name) and f.endswith(".pt") and not f.endswith("_optimizer.pt")),
                        key=lambda x: x[1], reverse=True)
        opts = sorted(((f, os.path.getmtime(os.path.join(self.checkpoint_dir, f))) for f in files
                       if f.startswith(name) and f.endswith("_optimizer.pt")), key=lambda x: x[1], reverse=True)
        pair = next(((m, o) for m, mt in models for o, ot in opts if abs(mt - ot) < 2), None)
        if pair is None:
            raise FileNotFoundError(f"Checkpoint {name} not found.")
        logger.info(f"Resuming training from {pair[0]} and {pair[1]}.")
        self.model.load_state_dict(torch.load(os.path.join(self.checkpoint_dir, pair[0]), weights_only=True))
        osd = torch.load(os.path.join(self.checkpoint_dir, pair[1]), weights_only=True)
        names = [n for n, _ in self.model.named_parameters()]
        vm, vv = self.model.plan.views(self._m), self.model.plan.views(self._v)
        t = 0.0
        for idx, st in osd.get("state", {}).items():
            n = names[int(idx)]
            vm[n].copy_(st["exp_avg"].to(vm[n].device))
            vv[n].copy_(st["exp_avg_sq"].to(vv[n].device))
            t = float(st["step"])
        self._state.copy_(torch.tensor([0.0, 1.0, t, 0.0]))
        self._fstate.copy_(torch.tensor([0.0, 1.0, t, 0.0, 0.0, 0.0, 0.0, 0.0] * 2))
        self._parity = 0

    def __call__(self, training: Any, **kwargs: Any) -> None:
        raise NotImplementedError()


class EvalPasses:
    """The validation and testing passes of train_epoch on the device
    (trainer.py:496-566), for HBM-resident embedding pools: every pass is the
    reference's batch loop (validation: ``validation_batches`` batches of
    (50 positives, 1,000 negatives), by default max(n_neg // 1000, n_pos // 50)
    as WakeWordTrainingDatasetIterator.validation's max_samples, training.py:
    693-701; testing: batches of (50 positives, 50 adversarial), max(n_pos // 50,
    n_adv // 50), :621-630) as ONE forward over all of its rows per pool
    (hbk_mlp_eval_count; the order of rows within a pass does not change its
    counts), with the input dropout on as in the reference (it never calls
    .eval()), then the bookkeeping of :509-536 / :549-561 and the dynamic
    negative weight on the device (hbk_mlp_eval_finish): no host
    synchronisation. Each pool is read in order with wrap-around, continuing
    where the previous pass stopped (the datasets' take() stream; a pass that
    covers whole laps of a pool reads every row equally often, as the
    reference's permutations do).

    Data-parallel (``group``, default the world): every rank evaluates a
    contiguous 1/W share of each pass's rows of its own pools, and the [2, 4]
    counts are summed with one all-reduce before the bookkeeping, so the
    false-positive rate, recall and the dynamic negative weight written into
    ``sched`` are the same on every rank (one global weight, as in the
    reference) and a pass costs each rank 1/W of its rows.

    ``run(sched, next_step)`` enqueues one validation (+ testing) pass on the
    current stream; the metrics land in ``history[k]`` = (false positives per
    hour, recall, testing false-positive rate, testing recall, testing
    accuracy, negative weight after, before, 0)."""

    def __init__(self, trainer: "WakeWordTrainer", validation_positive: torch.Tensor,
                 validation_negative: torch.Tensor, testing_positive: Optional[torch.Tensor] = None,
                 testing_adversarial: Optional[torch.Tensor] = None, validation_batch: Tuple[int, int] = (50, 1000),
                 testing_batch: Tuple[int, int] = (50, 50), validation_batches: Optional[int] = None,
                 testing_batches: Optional[int] = None,
                 target_false_positive_rate: float = DEFAULT_TARGET_FALSE_POSITIVE_RATE,
                 adjust_ratio: Optional[float] = DEFAULT_NEGATIVE_WEIGHT_ADJUST_RATIO,
                 activation_threshold: float = DEFAULT_ACTIVATION_THRESHOLD, seed: int = 0,
                 history_cap: int = 256, group: Optional["dist.ProcessGroup"] = None) -> None:
        self.trainer = trainer
        self.group = group
        dev = trainer.device
        pv, nv = validation_batch
        if validation_batches is None:
            validation_batches = max(validation_negative.shape[0] // nv, validation_positive.shape[0] // pv)
        # (pool, rows, label, counter set: 0 validation / 1 testing)
        self.parts = [(validation_positive, validation_batches * pv, 1, 0),
                      (validation_negative, validation_batches * nv, 0, 0)]
        self.sizes = [float(validation_batches * nv), float(validation_batches * pv), 0.0, 0.0]
        self.testing = testing_positive is not None and testing_adversarial is not None
        if self.testing:
            pt, at = testing_batch
            if testing_batches is None:
                testing_batches = max(testing_positive.shape[0] // pt, testing_adversarial.shape[0] // at)
            self.parts += [(testing_positive, testing_batches * pt, 1, 1),
                           (testing_adversarial, testing_batches * at, 0, 1)]
            self.sizes[2:] = [float(testing_batches * at), float(testing_batches * pt)]
        for pool, _, _, _ in self.parts:
            if pool.device != dev or pool.dtype not in (torch.float32, torch.float16) or not pool.is_contiguous():
                raise ValueError("evaluation pools must be contiguous f32 / f16 tensors on the trainer's device")
        self.offsets = [0] * len(self.parts)
        self.target = float(target_false_positive_rate)
        self.ratio = float(adjust_ratio) if adjust_ratio else 0.0
        self.act_thr = float(activation_threshold)
        self.seed = int(seed)
        plan = trainer.model.plan
        self.ws = torch.empty(plan.eval_workspace_bytes(max(r for _, r, _, _ in self.parts)), dtype=torch.uint8,
                              device=dev)
        self.counts = torch.zeros((2, 4), dtype=torch.float32, device=dev)
        self.history = torch.zeros((history_cap, 8), dtype=torch.float32, device=dev)
        self.side = os.environ.get("HBK_EVAL_SIDE", "0") == "1"  # the f32 pools on a side stream (run(); off)
        self._side_keep = None
        self.n = 0

    @property
    def rows_per_pass(self) -> int:
        return sum(r for _, r, _, _ in self.parts)

    def run_metrics(self) -> List[float]:
        """One pass (run() without a schedule), then its 8 metrics on the host:
        the train_epoch form (one device -> host read per validation step)."""
        saved, self.ratio = self.ratio, 0.0  # the caller applies the weight rule
        try:
            self.run()
        finally:
            self.ratio = saved
        return [float(v) for v in self.history[(self.n - 1) % self.history.shape[0]].tolist()]

    def run(self, sched: Optional[torch.Tensor] = None, next_step: int = 0) -> None:
        tr = self.trainer
        plan = tr.model.plan
        flat = tr.model.flat_parameters
        p = tr.model.dropout.p if tr.model.training else 0.0
        self.counts.zero_()
        plan.eval_prepare(flat, self.ws)
        # on a CU-masked stream (the pipelined train partition) the f32 pools' launches
        # (25 k rows each: a few rounds of workgroups, the last one partly empty) run on
        # a side stream with the same CU set, concurrently with the large f16 pool's, so
        # their workgroups fill each other's tails (64 CUs: 3.50 -> 3.43 ms per pass; on
        # the whole GPU it measured slower, so unmasked streams keep one queue); the
        # counts are atomics and the prepared weights are read-only here. Off by default
        # (HBK_EVAL_SIDE=1 turns it on): in the pipelined headline the extra queue cost
        # the featurize stream ~3 ms per 100 k-clip step (881 / 875 k against 857 / 853 k
        # clips/s, same box, alternating)
        cuda = self.trainer.device.type == "cuda"
        cur = torch.cuda.current_stream(self.trainer.device) if cuda else None
        side = None
        if cuda and self.side and any(pool.dtype == torch.float32 for pool, _, _, _ in self.parts):
            side, self._side_keep = capture_stream(self.trainer.device)
            if self._side_keep is None:  # not a CU-masked stream
                side = None
            else:
                side.wait_stream(cur)
        rank, world = distributed.world(self.group)
        # the f32 pools (validation positives, testing positives and adversarials: ~25 k rows
        # each) in ONE launch (hbk_mlp_eval_count_multi): each alone is ~3 rounds of workgroups
        # on a 64-CU stream run as 4; together their workgroups fill each other's last round
        multi = [] if (side is None and cuda and os.environ.get("HBK_EVAL_MULTI", "1") != "0") else None
        for k, (pool, rows, label, which) in enumerate(self.parts):
            # data-parallel: this rank's contiguous share of the pass's rows (the
            # shares partition the pass); the per-rank dropout stream differs
            lo, hi = distributed.clip_range(rows, rank, world)
            seed = (self.seed + 0x9E3779B97F4A7C15 * (self.n * 8 + k + 1) + 0xD1B54A32D192ED03 * rank) % (1 << 64)
            if multi is not None and pool.dtype == torch.float32 and hi > lo:
                multi.append((pool, hi - lo, (self.offsets[k] + lo) % pool.shape[0], label, which, seed))
            elif hi > lo:
                with torch.cuda.stream(side if side is not None and pool.dtype == torch.float32 else cur) \
                        if cuda else contextlib.nullcontext():
                    plan.eval_count(flat, pool, hi - lo, label, self.counts[which], self.ws,
                                    row_offset=(self.offsets[k] + lo) % pool.shape[0],
                                    activation_threshold=self.act_thr, dropout_p=p, seed=seed)
            self.offsets[k] = (self.offsets[k] + rows) % pool.shape[0]
        if multi:
            plan.eval_count_multi(flat, multi, self.counts, self.ws, activation_threshold=self.act_thr,
                                  dropout_p=p)
        if side is not None:
            cur.wait_stream(side)
        # one all-reduce of the [2, 4] counts: every rank computes the same rates and
        # the same next negative weight (the reference keeps one global weight)
        distributed.reduce_counts(self.counts, self.group)
        plan.eval_finish(self.counts[0], self.counts[1] if self.testing else None, self.sizes,
                         self.history[self.n % self.history.shape[0]], target=self.target, ratio=self.ratio,
                         sched=sched, next_step=next_step)
        self.n += 1


def _recall(tp: float, n_pos: float) -> float:
    return tp / n_pos if n_pos > 0 else 0.0


def _device_pools(it: Any) -> Optional[List[Tuple[torch.Tensor, int, int]]]:
    """[(rows [n, 1536] f32 / f16 on the device, per-batch count, label)] of a
    device-pool TrainingDatasetIterator (positives first, as next_batch), or None."""
    from heybuddy.dataset.training import DevicePool, TrainingDatasetIterator
    if not isinstance(it, TrainingDatasetIterator):
        return None
    try:
        it._pools()
    except (TypeError, ValueError):
        return None
    out = []
    for lst, lab in ((it.positive, 1), (it.negative, 0)):
        for d, n in lst:
            if not isinstance(d, DevicePool) or d.data.dtype not in (torch.float32, torch.float16):
                return None
            out.append((d, int(n), lab))
    return out


class _IndexedEpoch:
    """train_epoch over a device-pool iterator (the CLI's WakeWordTrainingDatasetIterator):
    the stage's batches drawn up front as pool indices (each dataset's take_indices(n x S):
    the rows and order of S next_batch() calls), labels, and the lr / negative-weight
    schedule on the device; the steps run as train_indexed segments (hipGraphs of 50
    steps, rows gathered on the device) up to each validation / checkpoint point, and
    validation / testing iterators become one EvalPasses over their pools. Same rows,
    same kernels and dropout stream as the per-batch loop (_step); HBK_TRAIN_EAGER=1 keeps
    the per-batch loop."""

    @classmethod
    def make(cls, tr: "WakeWordTrainer", training: Any, validation: Any, testing: Any, num_steps: int,
             threshold: float, act_thr: float, history: torch.Tensor) -> Optional["_IndexedEpoch"]:
        if not tr._fused or tr.device.type != "cuda" or os.environ.get("HBK_TRAIN_EAGER", "0") == "1":
            return None
        dsets = _device_pools(training)
        if dsets is None:
            return None
        if validation is not None and not isinstance(validation, EvalPasses):
            vd = _device_pools(validation)
            if vd is None or {lab for _, _, lab in vd} != {0, 1} or validation.max_samples is None:
                return None
        if testing is not None:
            td = _device_pools(testing)
            if (td is None or {lab for _, _, lab in td} != {0, 1} or testing.max_samples is None
                    or validation is None or isinstance(validation, EvalPasses)):
                return None
        return cls(tr, training, dsets, validation, testing, num_steps, threshold, act_thr, history)

    def __init__(self, tr, training, dsets, validation, testing, num_steps, threshold, act_thr, history):
        self.tr, self.threshold, self.act_thr, self.history = tr, threshold, act_thr, history
        dev = tr.device
        mx = training.max_samples
        self.S = num_steps if mx is None else min(num_steps, int(mx))
        p32, p16, off = tr._cat_pools([d.data for d, _, _ in dsets])
        cols, ys = [], []
        for d, n, lab in dsets:  # the S batches' rows, dataset by dataset (next_batch's column order)
            ix = d.take_indices(n * self.S).view(self.S, n).to(torch.int64) + off[id(d.data)]
            cols.append(ix if d.data.dtype == torch.float32 else -1 - ix)
            ys.append(torch.full((n,), float(lab), device=dev))
        training.total_yielded_samples += self.S
        idx, y = torch.cat(cols, 1), torch.cat(ys)
        self.batch = int(y.shape[0])
        rank, world = tr._world()
        if world > 1:  # distributed.shard_batch's class-stratified slice
            idx, y = idx[:, rank::world], y[rank::world]
        # the stage's index / label / schedule buffers persist per shape on the trainer, so the
        # next epoch's (and the next __call__'s) segments replay the hipGraphs captured now: the
        # graphs bake in these addresses, and a capture per stage per call cost ~20 ms of the
        # 3-stage bench run (bench.py's cli_path)
        idx = idx.to(torch.int32).contiguous()
        key = (tuple(idx.shape), str(dev))
        cache = getattr(tr, "_epoch_bufs", None)
        if cache is None:
            cache = tr._epoch_bufs = {}
        bufs = cache.get(key)
        if bufs is None:
            bufs = cache[key] = (torch.empty_like(idx), torch.empty_like(y),
                                          torch.zeros((max(self.S, 1), 2), dtype=torch.float32, device=dev))
        self.idx, self.y, self.sched = bufs
        self.idx.copy_(idx)
        self.y.copy_(y)
        self.sched.zero_()
        self.p32, self.p16 = p32, p16
        self.done = 0
        self.validation = validation
        if validation is not None and not isinstance(validation, EvalPasses):
            self.validation = tr._eval_from_iterators(validation, testing)

    def run_to(self, end: int, lr_hist: List[float], nw_hist: List[float]) -> None:
        """Steps done .. end - 1 (their lr / negative weights are in the host lists)."""
        if end <= self.done:
            return
        sc = torch.tensor(np.stack([np.asarray(lr_hist[self.done:end], np.float32),
                                    np.asarray(nw_hist[self.done:end], np.float32)], 1))
        self.sched[self.done:end].copy_(sc, non_blocking=False)
        self.tr.train_indexed(self.idx, self.y, self.sched, pool32=self.p32, pool16=self.p16,
                              threshold=self.threshold, activation_threshold=self.act_thr, history=self.history,
                              steps_per_graph=50, n_steps=end - self.done, continued=self.done > 0)
        self.done = end


class WakeWordTrainer(Trainer):
    """Trainer for the wake-word classifier (trainer.py:206-1007)."""

    def __init__(self, checkpoint_dir: str = "./checkpoints", learning_rate: float = DEFAULT_LEARNING_RATE,
                 input_shape: Tuple[int, int] = (16, 96), num_layers: int = DEFAULT_LAYERS,
                 layer_dim: int = DEFAULT_LAYER_DIM, num_heads: int = DEFAULT_HEADS,
                 architecture: str = DEFAULT_ARCHITECTURE, device: Optional[Union[str, torch.device]] = None,
                 **model_kwargs: Any) -> None:
        super().__init__(checkpoint_dir=checkpoint_dir, learning_rate=learning_rate, device=device,
                         input_shape=input_shape, num_layers=num_layers, layer_dim=layer_dim,
                         num_heads=num_heads, architecture=architecture, **model_kwargs)
        self.input_shape = input_shape
        self.num_layers = num_layers
        self.num_heads = num_heads
        self.architecture = architecture
        self.layer_dim = layer_dim

    def create_model(self, input_shape=(16, 96), architecture: str = DEFAULT_ARCHITECTURE,
                     layer_dim: int = DEFAULT_LAYER_DIM, num_layers: int = DEFAULT_LAYERS,
                     num_heads: int = DEFAULT_HEADS, **kwargs: Any) -> nn.Module:
        if architecture != "perceptron":
            raise NotImplementedError("the MI355X path implements the default 'perceptron' architecture")
        return WakeWordMLPModel(input_shape=input_shape, num_layers=num_layers, layer_dim=layer_dim, **kwargs)

    def num_false_positives(self, x: torch.Tensor, y: torch.Tensor,
                            activation_threshold: float = DEFAULT_ACTIVATION_THRESHOLD) -> torch.Tensor:
        return (y - x <= -activation_threshold).sum()

    def loss(self, x: torch.Tensor, y: torch.Tensor, weight: Optional[torch.Tensor] = None) -> torch.Tensor:
        if weight is None:
            return nn.functional.binary_cross_entropy(x, y)
        return nn.functional.binary_cross_entropy(x, y, weight.to(x.device))

    # -- data parallel ---------------------------------------------------------
    @staticmethod
    def _world() -> Tuple[int, int]:
        return distributed.world()

    def _step(self, x: torch.Tensor, y: torch.Tensor, lr: float, neg_weight: float, threshold: float,
              activation_threshold: float, history: Optional[torch.Tensor], seed: int) -> None:
        self._ensure_synced()
        rank, world = self._world()
        x, y = distributed.shard_batch(x, y, rank, world)
        dev = self.device
        x = x.to(dev, non_blocking=True)
        y = y.to(dev, non_blocking=True)
        plan = self.model.plan
        p = self.model.dropout.p if self.model.training else 0.0
        graphs = dev.type == "cuda" and os.environ.get("HBK_MLP_GRAPHS", "1") != "0"
        if self._fused:
            if graphs:
                self._fused_graph_step(x, y, lr, neg_weight, threshold, activation_threshold, history, p, world)
            else:
                xs = x.reshape(x.shape[0], -1).to(torch.float32).contiguous()
                ys = y.to(torch.float32).contiguous()
                plan.step_fwd_bwd(self.model.flat_parameters, self._bucket, self._fstate, self._parity, ys,
                                  xs.shape[0], pool32=xs, neg_weight=neg_weight, threshold=threshold,
                                  activation_threshold=activation_threshold, dropout_p=p, seed=self._seed_base)
                distributed.reduce_bucket(self._bucket)
                plan.step_update(self.model.flat_parameters, self._bucket, self._m, self._v, self._fstate,
                                 self._parity, lr=lr, beta1=BETAS[0], beta2=BETAS[1], eps=EPS, history=history)
            self._parity ^= 1
            return
        if graphs:
            self._graph_step(x, y, lr, neg_weight, threshold, activation_threshold, history,
                             seed * 1000003 + rank, p, world)
            return
        plan.train_fwd_bwd(self.model.flat_parameters, x.reshape(x.shape[0], -1), y, self._bucket,
                           neg_weight, threshold, activation_threshold, dropout_p=p,
                           seed=seed * 1000003 + rank)
        distributed.reduce_bucket(self._bucket)
        plan.gate_adam(self.model.flat_parameters, self._bucket, self._m, self._v, self._state, self._ctrl,
                       history, lr, BETAS[0], BETAS[1], EPS)

    @property
    def _seed_base(self) -> int:
        """Dropout stream of the fused path: fixed per trainer; every step adds
        its index and every epoch its salt (state[4]) on the device."""
        if not hasattr(self, "_seed_base_v"):
            self._seed_base_v = random.getrandbits(40)
        return self._seed_base_v

    def _fused_graph_step(self, x: torch.Tensor, y: torch.Tensor, lr: float, neg_weight: float,
                          threshold: float, activation_threshold: float, history: Optional[torch.Tensor],
                          p: float, world: int) -> None:
        """One fused step as captured hipGraphs, one set per (batch size, parity,
        thresholds, dropout p, history buffer). Each graph owns its staging rows,
        its (lr, neg_weight) cell and its workspace, so no later allocation can
        move memory a graph replays into. world == 1: one graph per step;
        data-parallel: forward/backward graph, all-reduce, update graph."""
        dev = self.device
        plan = self.model.plan
        flat = self.model.flat_parameters
        B = int(x.shape[0])
        key = (B, self._parity, float(threshold), float(activation_threshold), float(p), world,
               None if history is None else (history.data_ptr(), history.shape[0]), self._state_ptrs())
        g = self._graphs.get(key)
        if g is None:
            self._evict_graphs()
            sx = torch.zeros((B, plan.d_in), dtype=torch.float32, device=dev)
            sy = torch.zeros(B, dtype=torch.float32, device=dev)
            sched = torch.zeros((1, 2), dtype=torch.float32, device=dev)
            ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device=dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            parity = self._parity

            def fwd():
                plan.step_fwd_bwd(flat, self._bucket, self._fstate, parity, sy, B, pool32=sx, sched=sched,
                                  threshold=threshold, activation_threshold=activation_threshold, dropout_p=p,
                                  seed=self._seed_base, workspace=ws)

            def upd():
                plan.step_update(flat, self._bucket, self._m, self._v, self._fstate, parity, sched=sched,
                                 beta1=BETAS[0], beta2=BETAS[1], eps=EPS, history=history)

            graphs = []
            with torch.cuda.stream(side):
                if distributed.graph_capturable(world):  # one graph per step, the RCCL all-reduce inside
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=side):
                        fwd()
                        distributed.reduce_bucket(self._bucket)
                        upd()
                    graphs.append(gr)
                else:
                    for fn in (fwd, upd):
                        gr = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gr, stream=side):
                            fn()
                        graphs.append(gr)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = self._graphs[key] = {"x": sx, "y": sy, "sched": sched, "ws": ws, "graphs": graphs}
        g["x"].copy_(x.reshape(B, -1), non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        g["sched"][0, 0].fill_(float(lr))
        g["sched"][0, 1].fill_(float(neg_weight))
        if len(g["graphs"]) == 1:
            g["graphs"][0].replay()
        else:
            g["graphs"][0].replay()
            distributed.reduce_bucket(self._bucket)
            g["graphs"][1].replay()

    def train_indexed(self, idx: torch.Tensor, y: torch.Tensor, sched: torch.Tensor,
                      pool32: Optional[torch.Tensor] = None, pool16: Optional[torch.Tensor] = None,
                      threshold: float = DEFAULT_HIGH_LOSS_THRESHOLD,
                      activation_threshold: float = DEFAULT_ACTIVATION_THRESHOLD,
                      history: Optional[torch.Tensor] = None, steps_per_graph: int = 16,
                      graphs: bool = True, n_steps: Optional[int] = None, continued: bool = False) -> None:
        """S fused optimisation steps whose batches are rows of HBM-resident
        embedding pools (the device-side sampler's output): step s trains on
        rows idx[s] (int32 [S, B]; >= 0 -> pool32 f32 [n, 16, 96], < 0 ->
        pool16 f16 row -i-1) with labels y (f32 [B], the same composition every
        step, or [S, B]) at sched[s] = (lr, neg_weight). The step index lives on
        the device, so a hipGraph of ``steps_per_graph`` steps replays the whole
        run; continues from the current state (call _reset_accumulation() to
        start an epoch). ``n_steps``: run only this many of the steps (the rest
        in later calls, e.g. around an evaluation pass); ``continued``: the
        previous call ran the steps just before these on the same buffers, so
        its last step already gathered this call's first rows and kept the
        weight cache current. Data-parallel: every rank passes its own rows;
        one all-reduce of the bucket per step."""
        if not self._fused:
            raise NotImplementedError("train_indexed needs the fused train step (default architecture)")
        self._ensure_synced()
        dev = self.device
        plan = self.model.plan
        flat = self.model.flat_parameters
        S_all, B = int(idx.shape[0]), int(idx.shape[1])
        S = S_all if n_steps is None else int(n_steps)
        y_stride = B if y.dim() == 2 else 0
        p = self.model.dropout.p if self.model.training else 0.0
        p32 = None if pool32 is None else pool32.reshape(pool32.shape[0], -1)
        p16 = None if pool16 is None else pool16.reshape(pool16.shape[0], -1)
        _, world = self._world()
        ws = self._indexed_ws = getattr(self, "_indexed_ws", None)
        need = plan.workspace_bytes(B)
        if ws is None or ws.numel() < need or ws.device != dev:
            ws = self._indexed_ws = torch.empty(need, dtype=torch.uint8, device=dev)
            continued = False  # a new workspace holds no prefetched rows or weight cache

        # Each step also gathers + normalises the NEXT step's rows inside its own
        # launches (prefetch_next); only the first step of this call gathers its own.
        # One process: the weight-gradient slabs go straight to the update (no all-reduce between).
        defer = not distributed.reduces()

        # HBK_NO_PREFETCH=1 (A/B): every step gathers its own rows in a k1a launch
        pre = os.environ.get("HBK_NO_PREFETCH") is None

        def one(parity: int, ready: bool) -> None:
            plan.step_fwd_bwd(flat, self._bucket, self._fstate, parity, y, B, pool32=p32, pool16=p16, idx=idx,
                              idx_stride=B, y_stride=y_stride, sched=sched, threshold=threshold,
                              activation_threshold=activation_threshold, dropout_p=p, seed=self._seed_base,
                              workspace=ws, xhat_ready=ready and pre, prefetch_next=pre, idx_steps=S_all,
                              weights_ready=ready, defer_partials=defer)
            distributed.reduce_bucket(self._bucket)
            plan.step_update(flat, self._bucket, self._m, self._v, self._fstate, parity, sched=sched,
                             beta1=BETAS[0], beta2=BETAS[1], eps=EPS, history=history, workspace=ws)

        done = 0
        if S > 0:  # the first step gathers its own rows (unless continued) and prefetches the next
            one(self._parity, bool(continued))
            self._parity ^= 1
            done = 1
        k = max(2, steps_per_graph - steps_per_graph % 2)
        ptrs = tuple(t.data_ptr() if t is not None else 0 for t in (idx, y, sched, p32, p16, history, ws))
        ptrs += self._state_ptrs()

        def graph_of(n: int) -> "torch.cuda.CUDAGraph":
            """The captured graph of n (even) steps from the current parity."""
            key = ("indexed", n, self._parity, B, y_stride, float(threshold), float(activation_threshold), float(p),
                   defer, pre, ptrs, torch.cuda.current_stream(dev).cuda_stream)
            entry = self._graphs.get(key)
            if entry is not None:
                return entry[0]
            self._evict_graphs()
            side, keep = capture_stream(dev)  # the replay stream's CU mask, if any
            side.wait_stream(torch.cuda.current_stream(dev))
            gr = torch.cuda.CUDAGraph()
            par0 = self._parity
            with torch.cuda.stream(side):
                with torch.cuda.graph(gr, stream=side):
                    for j in range(n):
                        one(par0 ^ (j & 1), True)
            torch.cuda.current_stream(dev).wait_stream(side)
            self._graphs[key] = (gr, ws, keep)  # the entry keeps the baked-in workspace alive
            return gr

        if graphs and distributed.graph_capturable(world) and S - done >= 2:
            # k-step graphs, then one graph for the even remainder: at most one
            # more eager step (each eager step is ~1 ms of host time, a graph
            # replay a few us, and the host must stay ahead of the device).
            # Data-parallel on RCCL: every step's all-reduce is captured too.
            if S - done >= k:
                gr = graph_of(k)
                while S - done >= k:
                    gr.replay()
                    done += k
            tail = (S - done) - (S - done) % 2
            if tail >= 2:
                graph_of(tail).replay()
                done += tail
        while done < S:
            one(self._parity, True)
            self._parity ^= 1
            done += 1

    _MAX_GRAPHS = 16  # (a 3-stage call: ~2 step graphs per stage and parity, kept across calls)

    def _state_ptrs(self) -> tuple:
        """Addresses a captured step bakes in besides its own buffers: the flat
        parameters, Adam moments, gradient bucket and step state. Part of every
        graph key, so a re-flattened or moved model never replays into freed
        memory."""
        return tuple(t.data_ptr() for t in (self.model.flat_parameters, self._m, self._v, self._bucket,
                                            self._fstate))

    def _evict_graphs(self) -> None:
        """Bound the capture cache: each captured graph holds its staging
        buffers, workspace and memory pool, and the per-epoch keys (history
        buffer, stage batch size) would otherwise accumulate for the
        trainer's lifetime. Oldest captures go first."""
        while len(self._graphs) >= self._MAX_GRAPHS:
            self._graphs.pop(next(iter(self._graphs)))

    def _graph_step(self, x: torch.Tensor, y: torch.Tensor, lr: float, neg_weight: float, threshold: float,
                    activation_threshold: float, history: Optional[torch.Tensor], seed: int, p: float,
                    world: int) -> None:
        """The same step as two captured hipGraphs (forward/loss/backward, then gate +
        Adam; the all-reduce runs between them when world > 1). lr, neg_weight and
        the dropout seed change every step, so the kernels read them from a device
        float64 [3] (hbk_mlp_set_step_scalars) filled before each replay. One
        capture per (batch size, thresholds, dropout p, buffers): ~45 launches per
        step become 2 graph launches + 3 fills + the batch copies."""
        dev = self.device
        plan = self.model.plan
        flat = self.model.flat_parameters
        B = int(x.shape[0])
        key = (B, float(threshold), float(activation_threshold), float(p), world,
               tuple(t.data_ptr() for t in (flat, self._m, self._v, self._state, self._ctrl, self._bucket)),
               None if history is None else (history.data_ptr(), history.shape[0]))
        graphs = self._graphs
        g = graphs.get(key)
        if g is None:
            self._evict_graphs()
            if getattr(self, "_scalars", None) is None or self._scalars.device != dev:
                self._scalars = torch.zeros(3, dtype=torch.float64, device=dev)
            sx = torch.zeros((B, plan.d_in), dtype=torch.float32, device=dev)
            sy = torch.zeros(B, dtype=torch.float32, device=dev)
            # the graph owns its workspace: the plan's shared eager one may be
            # reallocated by a larger (validation) batch after the capture
            ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device=dev)
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            fwd, upd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            plan.set_step_scalars(self._scalars)
            try:
                with torch.cuda.graph(fwd, stream=side):
                    plan.train_fwd_bwd(flat, sx, sy, self._bucket, 1.0, threshold, activation_threshold,
                                       dropout_p=p, seed=0, workspace=ws)
                with torch.cuda.graph(upd, stream=side):
                    plan.gate_adam(flat, self._bucket, self._m, self._v, self._state, self._ctrl, history,
                                   1.0, BETAS[0], BETAS[1], EPS)
            finally:
                plan.set_step_scalars(None)  # eager launches keep their by-value arguments
            torch.cuda.current_stream(dev).wait_stream(side)
            g = graphs[key] = {"x": sx, "y": sy, "ws": ws, "fwd": fwd, "upd": upd}
        g["x"].copy_(x.reshape(B, -1), non_blocking=True)
        g["y"].copy_(y, non_blocking=True)
        self._scalars[0].fill_(float(lr))
        self._scalars[1].fill_(float(neg_weight))
        self._scalars[2].fill_(float(seed))  # < 2^53: exact in float64
        g["fwd"].replay()
        distributed.reduce_bucket(self._bucket)
        g["upd"].replay()

    @torch.no_grad()
    def _cat_pools(self, tensors: List[torch.Tensor]):
        """(pool32, pool16, {id(tensor): row offset}) for device datasets of both
        dtypes: each dtype's distinct tensors as [n, 1536] rows, concatenated once and
        cached (a single tensor of a dtype is used in place)."""
        key = tuple((id(t), t.data_ptr(), t.shape[0], t.dtype) for t in tensors)
        cache = getattr(self, "_pool_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        out: List[Optional[torch.Tensor]] = []
        off: Dict[int, int] = {}
        for dt in (torch.float32, torch.float16):
            uniq = list({id(t): t for t in tensors if t.dtype == dt}.values())
            o = 0
            for t in uniq:
                off[id(t)] = o
                o += int(t.shape[0])
            rows = [t.reshape(t.shape[0], -1) for t in uniq]
            out.append(None if not rows else rows[0].contiguous() if len(rows) == 1 else torch.cat(rows).contiguous())
        res = (out[0], out[1], off)
        self._pool_cache = (key, res)
        return res

    def _eval_from_iterators(self, validation: Any, testing: Any) -> "EvalPasses":
        """EvalPasses over device-pool validation / testing iterators (batches of
        their per-dataset counts, max_samples batches per pass; several datasets of a
        side are concatenated once)."""
        def side(it, label):
            ds = [(d.data, n) for d, n, lab in _device_pools(it) if lab == label]
            if not ds:
                return None, 0
            rows = [t.reshape(t.shape[0], -1) for t, _ in ds]
            dt = torch.float16 if all(t.dtype == torch.float16 for t in rows) else torch.float32
            pool = rows[0].contiguous() if len(rows) == 1 else torch.cat([r.to(dt) for r in rows]).contiguous()
            return pool, sum(n for _, n in ds)
        key = (id(validation), id(testing))
        cache = getattr(self, "_eval_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        vp, npv = side(validation, 1)
        vn, nnv = side(validation, 0)
        kw: Dict[str, Any] = {}
        if testing is not None:
            tp_, npt = side(testing, 1)
            ta, nat = side(testing, 0)
            if tp_ is not None and ta is not None:
                kw = dict(testing_positive=tp_, testing_adversarial=ta, testing_batch=(npt, nat),
                          testing_batches=testing.max_samples)
        ev = EvalPasses(self, vp, vn, validation_batch=(npv, nnv), validation_batches=validation.max_samples,
                        adjust_ratio=None, seed=random.getrandbits(31), **kw)
        self._eval_cache = (key, ev)
        return ev

    def _predict_all(self, data: Any) -> Tuple[torch.Tensor, torch.Tensor]:
        preds, labels = [], []
        for datum in data:
            x, y = datum[0].to(self.device), datum[1].to(self.device)
            preds.append(self.model(x)[:, 0])
            labels.append(y)
        return torch.cat(preds), torch.cat(labels)

    def train_epoch(self, training: Any, validation: Optional[Any] = None, testing: Optional[Any] = None,
                    num_steps: int = DEFAULT_STEPS, warmup_steps: int = DEFAULT_WARMUP_STEPS,
                    hold_steps: int = DEFAULT_HOLD_STEPS,
                    negative_weight_schedule: Union[float, List[float]] = DEFAULT_NEGATIVE_WEIGHT,
                    negative_weight_adjust_ratio: Optional[float] = None,
                    target_false_positive_rate: float = DEFAULT_TARGET_FALSE_POSITIVE_RATE,
                    validation_steps: int = DEFAULT_VALIDATION_STEPS,
                    checkpoint_steps: int = DEFAULT_CHECKPOINT_STEPS,
                    logging_steps: int = DEFAULT_LOGGING_STEPS,
                    learning_rate: float = DEFAULT_LEARNING_RATE,
                    high_loss_threshold: float = DEFAULT_HIGH_LOSS_THRESHOLD,
                    activation_threshold: float = DEFAULT_ACTIVATION_THRESHOLD,
                    description: str = "Training", name: str = "heybuddy", last_loss: float = 0.0,
                    last_recall: float = 0.0, last_false_positive_rate: float = 0.0,
                    last_validation_false_positive_per_hour: float = 0.0,
                    last_validation_recall: float = 0.0, last_testing_accuracy: float = 0.0,
                    last_testing_recall: float = 0.0, last_testing_false_positive_rate: float = 0.0,
                    use_wandb: bool = False) -> Tuple[Optional[torch.Tensor], ...]:
        """One epoch (trainer.py:314-608). Returns the reference's 11 histories.

        ``validation`` / ``testing``: iterables of (x, y) batches, evaluated by
        the HIP forward batch by batch (_predict_all: the CLI's dataset
        iterators), or ``validation`` an EvalPasses over HBM-resident pools
        (validation and testing in one device pass each, ``testing`` None)."""
        if use_wandb:
            logger.warning("wandb logging is outside the MI355X hot path; ignored")
        if isinstance(validation, EvalPasses) and testing is not None:
            raise ValueError("train_epoch: with an EvalPasses validation the testing pass runs from its "
                             "testing pools (EvalPasses(..., testing=...)); pass testing=None")
        self._reset_accumulation(salt=random.getrandbits(24))
        cap = getattr(self, "_history", None)
        if cap is None or cap.shape[0] < num_steps or cap.device != self.device:
            self._history = torch.zeros((max(num_steps, 1), 8), dtype=torch.float32, device=self.device)
            self._graphs = {k: v for k, v in self._graphs.items() if k[0] == "indexed"}
        history = self._history
        history.zero_()
        lr_hist: List[float] = []
        nw_hist: List[float] = []
        batch_sizes: List[int] = []
        v_fp: List[float] = []
        v_rec: List[float] = []
        t_acc: List[float] = []
        t_rec: List[float] = []
        t_fp: List[float] = []
        seed0 = random.getrandbits(31)
        # device-pool iterators (the CLI's): the stage as device-sampled indexed steps in
        # hipGraph segments (train_indexed) between the validation / checkpoint points, the
        # validation and testing iterators as device evaluation passes (EvalPasses)
        fast = _IndexedEpoch.make(self, training, validation, testing, num_steps, high_loss_threshold,
                                  activation_threshold, history)
        lr_all = None
        if fast is not None:
            validation, testing = fast.validation, None
            # the stage's schedule in one vectorised call (the same numpy ufuncs, bit-identical
            # values; ~6.5 us of host time per step when evaluated step by step)
            lr_all = self.get_learning_rate(np.arange(max(num_steps, 1)), warmup_steps=warmup_steps,
                                            hold_steps=hold_steps, total_steps=num_steps,
                                            target_learning_rate=learning_rate)
        for step, datum in enumerate(training) if fast is None else enumerate(range(fast.S)):
            if step >= num_steps:
                break
            if fast is None:
                x, y = datum[0], datum[1]
            lr = float(self.get_learning_rate(step, warmup_steps=warmup_steps, hold_steps=hold_steps,
                                              total_steps=num_steps, target_learning_rate=learning_rate)
                       if lr_all is None else lr_all[step])
            lr_hist.append(lr)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
            if isinstance(negative_weight_schedule, (float, int)):
                nw = float(negative_weight_schedule)
            elif len(negative_weight_schedule) <= step:
                nw = float(negative_weight_schedule[-1])
            else:
                nw = float(negative_weight_schedule[step])
            nw_hist.append(nw)
            if fast is None:
                batch_sizes.append(int(y.shape[0]))
                self._step(x, y, lr, nw, high_loss_threshold, activation_threshold, history, seed0 + step)
            else:
                batch_sizes.append(fast.batch)
                if step > 0 and ((validation is not None and step % validation_steps == 0)
                                 or step % checkpoint_steps == 0):
                    fast.run_to(step + 1, lr_hist, nw_hist)
            if step > 0 and step % validation_steps == 0:
                if isinstance(validation, EvalPasses):
                    # HBM-resident pools: the passes on the device (hbk_mlp_eval_*), one
                    # host read of the pass's 8 metrics; the weight rule stays on the host
                    vals = validation.run_metrics()
                    fph = vals[0]
                    v_fp.append(fph)
                    v_rec.append(vals[1])
                    if validation.testing:
                        t_fp.append(vals[2])
                        t_rec.append(vals[3])
                        t_acc.append(vals[4])
                    if negative_weight_adjust_ratio is not None:
                        assert isinstance(negative_weight_schedule, float), \
                            "Negative weight schedule must be a float when using dynamic negative weight adjustment."
                        if fph > target_false_positive_rate:
                            negative_weight_schedule = negative_weight_schedule * negative_weight_adjust_ratio
                        else:
                            negative_weight_schedule = max(1.0, negative_weight_schedule / negative_weight_adjust_ratio)
                elif validation is not None:
                    preds, labels = self._predict_all(validation)
                    n_neg = int((labels == 0).sum().item())
                    hours = n_neg * 1.44 / 3600
                    n_fp = float(self.num_false_positives(preds, labels, activation_threshold).item())
                    # torch tensor division in the reference (trainer.py:511): x / 0 -> inf (nan for 0 / 0)
                    fph = n_fp / hours if hours > 0 else (float("inf") if n_fp > 0 else float("nan"))
                    v_fp.append(fph)
                    pos = labels == 1
                    v_rec.append(_recall(float((preds[pos] > activation_threshold).sum().item()),
                                         float(pos.sum().item())))
                    if negative_weight_adjust_ratio is not None:
                        assert isinstance(negative_weight_schedule, float), \
                            "Negative weight schedule must be a float when using dynamic negative weight adjustment."
                        if fph > target_false_positive_rate:
                            negative_weight_schedule = negative_weight_schedule * negative_weight_adjust_ratio
                        else:
                            negative_weight_schedule = max(1.0, negative_weight_schedule / negative_weight_adjust_ratio)
                if testing is not None and not isinstance(validation, EvalPasses):
                    preds, labels = self._predict_all(testing)
                    n_neg = max(int((labels == 0).sum().item()), 1)
                    t_fp.append(float(self.num_false_positives(preds, labels, activation_threshold).item()) / n_neg)
                    pos = labels == 1
                    t_rec.append(_recall(float((preds[pos] > activation_threshold).sum().item()),
                                         float(pos.sum().item())))
                    t_acc.append(float(((preds > activation_threshold).float() == labels.float()).float().mean().item()))
            elif v_fp or t_acc:
                if validation is not None:
                    v_fp.append(v_fp[-1])
                    v_rec.append(v_rec[-1])
                if testing is not None or (isinstance(validation, EvalPasses) and validation.testing):
                    t_fp.append(t_fp[-1])
                    t_rec.append(t_rec[-1])
                    t_acc.append(t_acc[-1])
            else:
                if validation is not None:
                    v_fp.append(last_validation_false_positive_per_hour)
                    v_rec.append(last_validation_recall)
                if testing is not None or (isinstance(validation, EvalPasses) and validation.testing):
                    t_fp.append(last_testing_false_positive_rate)
                    t_rec.append(last_testing_recall)
                    t_acc.append(last_testing_accuracy)
            if step > 0 and step % checkpoint_steps == 0:
                self.save_checkpoint(f"{name}_{step}")
        if fast is not None:
            fast.run_to(len(lr_hist), lr_hist, nw_hist)
        n_steps = len(lr_hist)
        h = history[:n_steps].cpu().numpy().astype(np.float64)
        loss_h, rec_h, fp_h, hlr_h = self._rebuild_histories(h, batch_sizes, last_loss, last_recall,
                                                             last_false_positive_rate)

        def T(v):
            return torch.tensor(v, dtype=torch.float64) if v else None

        return (T(lr_hist), T(nw_hist), T(loss_h), T(hlr_h), T(rec_h), T(fp_h), T(v_fp), T(v_rec),
                T(t_acc), T(t_rec), T(t_fp))

    @staticmethod
    def _rebuild_histories(h: np.ndarray, batch_sizes: List[int], last_loss: float, last_recall: float,
                           last_fp: float):
        """The reference's per-step bookkeeping (trainer.py:443-494) from the
        device record [n_sel, acc_steps, fired, loss, n_neg, fp, n_pos, tp]."""
        loss_h: List[float] = []
        rec_h: List[float] = []
        fp_h: List[float] = []
        hlr_h: List[float] = []
        acc = None  # accumulated (n_neg, fp, n_pos, tp) of the pending predictions
        for k, row in enumerate(h):
            n_sel, _, fired, loss, n_neg, fp, n_pos, tp = row
            hlr_h.append(n_sel / batch_sizes[k])
            cur = np.array([n_neg, fp, n_pos, tp])
            if n_sel > 0:
                if n_sel >= 128:
                    acc = cur
                if fired == 0:
                    acc = cur if acc is None else acc + cur
                    if loss_h:
                        loss_h.append(loss_h[-1])
                        rec_h.append(rec_h[-1])
                        fp_h.append(fp_h[-1])
                else:
                    a = acc if acc is not None else np.zeros(4)
                    loss_h.append(float(loss))
                    rec_h.append(_recall(a[3], a[2]))
                    fp_h.append(a[1] / max(a[0], 1.0))
                    acc = None
            elif loss_h:
                loss_h.append(loss_h[-1])
                rec_h.append(rec_h[-1])
                fp_h.append(fp_h[-1])
            else:
                loss_h.append(last_loss)
                rec_h.append(last_recall)
                fp_h.append(last_fp)
        return loss_h, rec_h, fp_h, hlr_h

    def __call__(self, training: Any, validation: Optional[Any] = None, testing: Optional[Any] = None,
                 num_steps: int = DEFAULT_STEPS, num_stages: int = DEFAULT_STAGES,
                 max_negative_weight: float = DEFAULT_NEGATIVE_WEIGHT,
                 logging_steps: int = DEFAULT_LOGGING_STEPS, validation_steps: int = DEFAULT_VALIDATION_STEPS,
                 checkpoint_steps: int = DEFAULT_CHECKPOINT_STEPS,
                 target_false_positive_rate: float = DEFAULT_TARGET_FALSE_POSITIVE_RATE,
                 negative_weight_adjust_ratio: float = DEFAULT_NEGATIVE_WEIGHT_ADJUST_RATIO,
                 dynamic_negative_weight: bool = DEFAULT_DYNAMIC_NEGATIVE_WEIGHT,
                 batch_size_adjust_ratio: float = DEFAULT_BATCH_SIZE_ADJUST_RATIO,
                 learning_rate_adjust_ratio: float = DEFAULT_LEARNING_RATE_ADJUST_RATIO,
                 step_adjust_ratio: float = DEFAULT_STEP_ADJUST_RATIO,
                 learning_rate: float = DEFAULT_LEARNING_RATE,
                 high_loss_threshold: float = DEFAULT_HIGH_LOSS_THRESHOLD,
                 activation_threshold: float = DEFAULT_ACTIVATION_THRESHOLD,
                 wandb_entity: Optional[str] = None, name: str = "heybuddy", **kwargs: Any) -> Dict[str, Any]:
        """3-stage training (trainer.py:764-1007): after each stage lr x 0.5,
        steps x 2 (at least validation_steps), batch x 0.5, and the last
        validated negative weight carries over."""
        start = perf_counter()
        hist: Dict[str, List[torch.Tensor]] = {k: [] for k in ("lr", "nw", "loss", "hlr", "recall", "fp", "vfp",
                                                               "vrecall", "tacc", "trecall", "tfp")}
        last = {"loss": 0.0, "recall": 0.0, "fp": 0.0, "vfp": 0.0, "vrec": 0.0, "tacc": 0.0, "trec": 0.0, "tfp": 0.0}
        for hook in ("start",):
            for d in (training, validation, testing):
                if hasattr(d, hook):
                    getattr(d, hook)()
        # the per-step history buffer sized once for the longest stage: train_indexed's hipGraphs
        # bake in its address, so a buffer regrown by a later stage made every stage of the next
        # call capture its graphs again (6 captures, ~28 ms of a 3-stage bench call)
        n_max, n_ = num_steps, num_steps
        for _ in range(num_stages - 1):
            n_ = max(validation_steps, int(n_ * step_adjust_ratio))
            n_max = max(n_max, n_)
        cap = getattr(self, "_history", None)
        if cap is None or cap.shape[0] < n_max or cap.device != self.device:
            self._history = torch.zeros((max(n_max, 1), 8), dtype=torch.float32, device=self.device)
        for i in range(num_stages):
            if dynamic_negative_weight:
                weights: Union[float, List[float]] = max_negative_weight
                ratio: Optional[float] = negative_weight_adjust_ratio
            else:
                weights = np.linspace(1, max_negative_weight, num_steps).tolist()
                ratio = None
            t0 = perf_counter()
            lr, nw, loss, hlr, rec, fp, v_fp, v_rec, t_acc, t_rec, t_fp = self.train_epoch(
                training, validation=validation, testing=testing, num_steps=num_steps,
                negative_weight_schedule=weights, negative_weight_adjust_ratio=ratio,
                target_false_positive_rate=target_false_positive_rate, learning_rate=learning_rate,
                warmup_steps=num_steps // 5, hold_steps=num_steps // 3, logging_steps=logging_steps,
                validation_steps=validation_steps, checkpoint_steps=checkpoint_steps,
                description=f"Training Stage {i + 1}", high_loss_threshold=high_loss_threshold,
                activation_threshold=activation_threshold, name=f"{name}_{i}", last_loss=last["loss"],
                last_recall=last["recall"], last_false_positive_rate=last["fp"],
                last_validation_false_positive_per_hour=last["vfp"], last_validation_recall=last["vrec"],
                last_testing_accuracy=last["tacc"], last_testing_recall=last["trec"],
                last_testing_false_positive_rate=last["tfp"])
            logger.info(f"Training Stage {i + 1}: {len(lr)} steps in {perf_counter() - t0:.2f} s, "
                        f"final loss {float(loss[-1]) if loss is not None else float('nan'):.5f}")
            for k, v in zip(("lr", "nw", "loss", "hlr", "recall", "fp", "vfp", "vrecall", "tacc", "trecall", "tfp"),
                            (lr, nw, loss, hlr, rec, fp, v_fp, v_rec, t_acc, t_rec, t_fp)):
                if v is not None:
                    hist[k].append(v)
            last.update(loss=float(loss[-1]), recall=float(rec[-1]), fp=float(fp[-1]))
            if v_fp is not None:
                last.update(vfp=float(v_fp[-1]), vrec=float(v_rec[-1]))
            if t_acc is not None:
                last.update(tacc=float(t_acc[-1]), trec=float(t_rec[-1]), tfp=float(t_fp[-1]))
            learning_rate *= learning_rate_adjust_ratio
            num_steps = max(validation_steps, int(num_steps * step_adjust_ratio))
            if v_fp is not None and dynamic_negative_weight:
                max_negative_weight = float(nw[-1])
            if hasattr(training, "multiply_batch_size"):
                training.multiply_batch_size(batch_size_adjust_ratio)
        self.save_checkpoint(f"{name}_final")
        for d in (training, validation, testing):
            if hasattr(d, "stop"):
                d.stop()
        logger.info(f"Training complete in {perf_counter() - start:.2f} s")
        return {k: torch.cat(v) for k, v in hist.items() if v}
