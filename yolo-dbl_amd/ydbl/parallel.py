"""Batch-sharded multi-GPU inference: one process per GPU, one all-gather of the fixed-shape boxes.

The path partitions by image: rank r runs forward + decode + NMS on its contiguous
slice of the global batch into ``det[B_local, max_det, 6]`` + ``count[B_local]``; the only exchange is
one all-gather of those buffers (RCCL over xGMI with the "nccl" backend, gloo on CPU in the tests),
which assembles the detections in global batch order.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(global_batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, stop) slice of the global batch owned by ``rank`` (sizes differ by <= 1)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_detections(det: torch.Tensor, count: torch.Tensor, global_batch: int, group=None):
    """All-gather every rank's ``det [b_r, max_det, 6]`` / ``count [b_r]`` into global batch order.

    Ranks may own different numbers of images (``shard_bounds``); buffers are padded to the largest
    slice so the collective is a single fixed-shape all-gather per tensor.
    Returns (det_all [global_batch, max_det, 6], count_all [global_batch]) on every rank.
    """
    world = dist.get_world_size(group)
    b_max = -(-global_batch // world)
    b_loc = det.shape[0]
    if b_loc < b_max:
        det = torch.cat([det, det.new_zeros((b_max - b_loc,) + tuple(det.shape[1:]))])
        count = torch.cat([count, count.new_zeros(b_max - b_loc)])
    dets = [torch.empty_like(det) for _ in range(world)]
    cnts = [torch.empty_like(count) for _ in range(world)]
    dist.all_gather(dets, det.contiguous(), group=group)
    dist.all_gather(cnts, count.contiguous(), group=group)
    out_d, out_c = [], []
    for r in range(world):
        s, e = shard_bounds(global_batch, world, r)
        out_d.append(dets[r][: e - s])
        out_c.append(cnts[r][: e - s])
    return torch.cat(out_d), torch.cat(out_c)


def detections_list(det_all: torch.Tensor, count_all: torch.Tensor):
    """[n_i, 6] per image (one host sync)."""
    cnt = count_all.tolist()
    return [det_all[i, : cnt[i]] for i in range(det_all.shape[0])]


class ShardedPredictor:
    """Runs a model's compiled session on this rank's slice and returns global detections."""

    def __init__(self, model, global_batch: int, h: int, w: int, device, group=None, **session_kw):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.group = group
        self.global_batch = global_batch
        self.start, self.stop = shard_bounds(global_batch, self.world, self.rank)
        self.session = model.session(self.stop - self.start, h, w, device=device, **session_kw)

    def __call__(self, images_global: torch.Tensor | None = None, images_local: torch.Tensor | None = None):
        x = images_local if images_local is not None else images_global[self.start:self.stop]
        det, cnt = self.session(x)
        if self.world == 1:
            return det, cnt
        return gather_detections(det, cnt, self.global_batch, self.group)
