"""Data-parallel inference over the GPUs of one node.

Images are independent through the whole forward (no batch statistics, LayerNorm per
token), so a global batch is split into contiguous per-rank shards, every rank runs the
replicated model on its shard, and the only exchange is one all-gather of the
(B_local, 17, 6) detections — RCCL over xGMI with backend "nccl", gloo on CPU for tests.
One process per GPU (torch.distributed.run); nothing here is CUDA-specific.

The reference is single-device (`ipynb:12`, no tf.distribute anywhere); this module is the
MI355X-side addition the north_star asks for.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, rank: int, world: int):
    """Contiguous shard [start, stop) of rank `rank`; the first `global_batch % world`
    ranks get one extra image (ragged batches are allowed)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(int(global_batch), world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def max_shard(global_batch: int, world: int) -> int:
    return -(-int(global_batch) // world)


def broadcast_weights(model, src: int = 0, group=None) -> None:
    """Make every replica hold rank `src`'s weights (e.g. after rank 0 loaded a
    checkpoint): broadcast the fp32 master tensors, then re-pack on each rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    backend = dist.get_backend(group)
    dev = model.device if backend == "nccl" else torch.device("cpu")
    names = model.weight_names()
    cur = model.get_weight_dict()
    out = {}
    for n in names:
        t = torch.as_tensor(cur[n]).to(dev).contiguous()
        dist.broadcast(t, src=src, group=group)
        out[n] = t.cpu()
    model.set_weights(out)


def gather_padded(padded: torch.Tensor, group=None) -> torch.Tensor:
    """The collective: every rank's equally sized `padded` shard, concatenated in rank
    order (one all_gather_into_tensor on RCCL; a list all_gather on gloo)."""
    world = dist.get_world_size(group)
    out = torch.empty((world * padded.shape[0],) + tuple(padded.shape[1:]), dtype=padded.dtype,
                      device=padded.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, padded.contiguous(), group=group)
    else:
        dist.all_gather(list(out.chunk(world)), padded.contiguous(), group=group)
    return out


def all_gather_detections(local: torch.Tensor, global_batch: int, group=None) -> torch.Tensor:
    """Gather every rank's (b_r, 17, 6) fp32 shard into (global_batch, 17, 6) in rank
    order.  Shards are padded to the largest shard so one fixed-size collective suffices
    (a single all_gather_into_tensor on RCCL)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ms = max_shard(global_batch, world)
    start, stop = shard_bounds(global_batch, rank, world)
    if local.shape[0] != stop - start:
        raise ValueError(f"rank {rank}: local shard has {local.shape[0]} rows, expected "
                         f"{stop - start}")
    if world == 1:
        return local
    padded = local
    if local.shape[0] != ms:
        padded = torch.zeros((ms,) + tuple(local.shape[1:]), dtype=local.dtype,
                             device=local.device)
        padded[:local.shape[0]] = local
    out = gather_padded(padded, group)
    pieces = [out[r * ms: r * ms + (shard_bounds(global_batch, r, world)[1] -
                                   shard_bounds(global_batch, r, world)[0])]
              for r in range(world)]
    return torch.cat(pieces, 0)


class DataParallelDetector:
    """Runs `forward_fn(images_shard) -> (b_r, 17, 6)` on this rank's shard of a global
    batch and all-gathers the detections.  `forward_fn` defaults to the replicated
    model's fused forward + decode (`Model.detect`, returning decoded detections)."""

    def __init__(self, model=None, forward_fn: Optional[Callable] = None, group=None):
        if forward_fn is None:
            if model is None:
                raise ValueError("need a model or a forward_fn")
            forward_fn = lambda x: model.detect(x)[1]
        self.forward_fn = forward_fn
        self.group = group

    def __call__(self, global_images: torch.Tensor) -> torch.Tensor:
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        rank = dist.get_rank(self.group) if dist.is_initialized() else 0
        b = global_images.shape[0]
        start, stop = shard_bounds(b, rank, world)
        local = self.forward_fn(global_images[start:stop])
        if world == 1:
            return local
        return all_gather_detections(local, b, self.group)

    def run_local(self, local_images: torch.Tensor, global_batch: int) -> torch.Tensor:
        """Variant for inputs that already live on their rank (bench / data loaders)."""
        local = self.forward_fn(local_images)
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return local
        return all_gather_detections(local, global_batch, self.group)
