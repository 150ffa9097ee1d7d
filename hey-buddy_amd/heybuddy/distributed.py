"""Data parallelism for the hot path (one process per GPU, torch.distributed;
backend "nccl" = RCCL over xGMI on the MI355X box, "gloo" in CPU tests).

* Featurization shards the clips: rank r owns clips [r N/W, (r+1) N/W); no
  collective on the data path.
* The classifier train step has ONE exchange: every rank trains on a
  class-stratified 1/W slice of each global batch (batches are
  [positives | adversarial | negatives], so a stride-W slice keeps the mix),
  and the unnormalised gradient bucket (256,417 grads + 8 statistics,
  1,025,700 B) is summed with a single all-reduce. The accumulation gate and
  the 1/(n_sel * accumulation_steps) normalisation then use the GLOBAL
  statistics, so every rank applies the identical Adam update and the result
  equals single-process training on the whole batch (§8e-2).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def world(group: Optional[dist.ProcessGroup] = None) -> Tuple[int, int]:
    """(rank, world size) in ``group`` (default the world); (0, 1) when
    torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def clip_range(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous clip shard of a rank (covers [0, n) exactly once)."""
    return (n * rank) // world_size, (n * (rank + 1)) // world_size


def shard_batch(x: torch.Tensor, y: torch.Tensor, rank: int, world_size: int):
    """Class-stratified slice of a global batch for one rank."""
    if world_size == 1:
        return x, y
    return x[rank::world_size], y[rank::world_size]


def force_reduce() -> bool:
    """HBK_DP_REDUCE_ALWAYS=1: run the bucket all-reduce even on a one-rank
    group (a single-GPU check that the RCCL call captures into the train
    step's hipGraph and replays; the sum over one rank is the identity)."""
    return os.environ.get("HBK_DP_REDUCE_ALWAYS") == "1" and dist.is_available() and dist.is_initialized()


def graph_capturable(world_size: int) -> bool:
    """Can the train step's all-reduce be captured into its hipGraph? RCCL
    (backend "nccl") collectives can be stream-captured; gloo stages through
    the host and cannot. HBK_DP_GRAPHS=0 forces the eager per-step path."""
    if world_size == 1 and not force_reduce():
        return True
    if os.environ.get("HBK_DP_GRAPHS", "1") == "0":
        return False
    return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"


def reduces(group: Optional[dist.ProcessGroup] = None) -> bool:
    """Does reduce_bucket run a collective here?"""
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size(group) > 1 or force_reduce())


def reduce_bucket(bucket: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Sum the gradient + statistics bucket over the data-parallel ranks (one
    all-reduce of the 1,025,700-B bucket; capturable into a hipGraph on RCCL)."""
    if reduces(group):
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    return bucket


def reduce_counts(counts: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Sum the evaluation passes' prediction counts over the ranks (in place;
    float32 counts are exact below 2^24 rows). No-op on one rank."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def broadcast_(t: torch.Tensor, src: int = 0, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Overwrite t with rank src's copy on every rank of ``group`` (in place; a
    device tensor goes through the host on gloo). No-op without a process
    group."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return t
    if dist.get_backend(group) == "gloo" and t.device.type != "cpu":
        h = t.detach().cpu()
        dist.broadcast(h, src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src, group=group)
    return t
