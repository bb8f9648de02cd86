"""Batch-sharded multi-GPU inference: one process per GPU, ONE all-gather of the fixed-shape boxes.

The path partitions by image: rank r runs forward + decode + NMS on its contiguous
slice of the global batch.  Its NMS writes straight into a per-image record buffer
``records [b_max, record_width(max_det)]`` fp32 = ``[det (max_det*6) | count (int32 bits) | pad]``
(ydbl_nms out_stride / count_stride), so the only exchange is one ``all_gather_into_tensor`` of that
buffer into a preallocated ``[world * b_max, width]`` buffer (RCCL over xGMI with the "nccl" backend,
gloo on CPU in the tests).  When every rank owns b_max images the gathered rows ARE the global batch in
order and the (det, count) results are views of them -- no concatenation, no copy.  The process group
follows the reference's DDP setup (U/engine/trainer.py:222-227: one process per device, backend
"nccl", rank / world size from the launcher's environment).
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


def record_width(max_det: int) -> int:
    """fp32 words per image record: max_det * 6 box words + 1 count word, padded to 16 bytes."""
    return (max_det * 6 + 1 + 3) // 4 * 4


def record_views(records: torch.Tensor, max_det: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(det [n, max_det, 6] fp32, count [n] int32) views of a [n, record_width] fp32 record buffer."""
    n, width = records.shape
    if width != record_width(max_det) or records.dtype != torch.float32 or records.stride(1) != 1:
        raise ValueError(f"not a record buffer for max_det {max_det}: {tuple(records.shape)} {records.dtype}")
    det = records[:, : max_det * 6].unflatten(1, (max_det, 6))
    count = records.view(torch.int32)[:, max_det * 6]
    return det, count


def gather_records(records: torch.Tensor, out: torch.Tensor, group=None) -> torch.Tensor:
    """The path's one collective: every rank's [b_max, width] records into out [world * b_max, width].  On a gloo
    group with device tensors (ranks sharing a GPU, e.g. the world-2 GPU test) the records go through host memory."""
    if records.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(host, records.cpu(), group=group)
        out.copy_(host)
        return out
    dist.all_gather_into_tensor(out, records, group=group)
    return out


class GlobalDetections:
    """Global-batch-order (det, count) over a gathered record buffer of `world` ranks x `b_max` rows."""

    def __init__(self, gathered: torch.Tensor, global_batch: int, world: int, max_det: int):
        self.gathered, self.global_batch, self.world, self.max_det = gathered, global_batch, world, max_det
        b_max = gathered.shape[0] // world
        if b_max * world == global_batch:
            self.rows = None  # every rank full: the gathered rows are the global batch
        else:  # ragged last ranks: their padding rows are skipped (one index_select when asked for)
            rows = [r * b_max + i for r in range(world) for i in range(shard_bounds(global_batch, world, r)[1]
                                                                          - shard_bounds(global_batch, world, r)[0])]
            self.rows = torch.tensor(rows, dtype=torch.long, device=gathered.device)

    def tensors(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(det_all [global_batch, max_det, 6], count_all [global_batch])."""
        g = self.gathered if self.rows is None else self.gathered.index_select(0, self.rows)
        return record_views(g, self.max_det)


def gather_detections(records: torch.Tensor, global_batch: int, max_det: int = 300, group=None):
    """One-shot form: all-gather this rank's record buffer (b_max rows, b_max = ceil(global_batch / world)) and
    return (det_all [global_batch, max_det, 6], count_all [global_batch]) in global batch order on every rank."""
    world = dist.get_world_size(group)
    out = records.new_empty((world * records.shape[0], records.shape[1]))
    gather_records(records, out, group)
    return GlobalDetections(out, global_batch, world, max_det).tensors()


def detections_list(det_all: torch.Tensor, count_all: torch.Tensor):
    """[n_i, 6] per image (one host sync)."""
    cnt = count_all.tolist()
    return [det_all[i, : cnt[i]] for i in range(det_all.shape[0])]


class ShardedPredictor:
    """This rank's slice of a global batch through a compiled session whose NMS writes the record buffer, then
    the one all-gather into a preallocated global buffer.  Without an initialised process group it is the
    plain session (world 1, no collective)."""

    def __init__(self, model, global_batch: int, h: int, w: int, device, group=None, max_det: int = 300,
                 **session_kw):
        self.distributed = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.group, self.global_batch, self.max_det = group, global_batch, max_det
        self.start, self.stop = shard_bounds(global_batch, self.world, self.rank)
        self.b_max = -(-global_batch // self.world)
        self.session = model.session(self.stop - self.start, h, w, device=device, max_det=max_det,
                                     gather_rows=self.b_max, **session_kw)
        self.records = self.session.records
        self.gathered = torch.empty((self.world * self.b_max, self.records.shape[1]), dtype=torch.float32,
                                    device=self.records.device)
        self.global_dets = GlobalDetections(self.gathered, global_batch, self.world, max_det)

    def load(self, images_global: torch.Tensor | None = None, images_local: torch.Tensor | None = None):
        x = images_local if images_local is not None else images_global[self.start:self.stop]
        self.session.load(x)

    def run(self):
        """Forward + decode + NMS of the loaded slice, then the all-gather (no host sync, no allocation)."""
        self.session.launch()
        if self.distributed:
            gather_records(self.records, self.gathered, self.group)

    def __call__(self, images_global: torch.Tensor | None = None, images_local: torch.Tensor | None = None):
        """(det_all [global_batch, max_det, 6], count_all [global_batch]) on every rank."""
        if images_global is not None or images_local is not None:
            self.load(images_global, images_local)
        self.run()
        if not self.distributed:
            return self.session.det, self.session.count
        return self.global_dets.tensors()
