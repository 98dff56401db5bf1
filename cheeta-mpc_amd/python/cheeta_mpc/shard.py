"""Multi-GPU sharding of a QP batch: one process per GPU, contiguous QP-id ranges, no data-path
collective. The counter-based generator keys every QP's inputs by its global id, so a QP's inputs and solution are
the same whatever the number of ranks; torch.distributed (gloo) is used only for barriers and the max-over-ranks
time."""
import os


def shard_range(total, world, rank):
    """Contiguous [offset, offset+count) slice of `total` QPs for `rank` of `world` (sizes differ by at most 1)."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


class Dist:
    """Thin wrapper over torch.distributed (gloo) for barriers and scalar reductions; a no-op at world size 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self._d = None
        if self.world > 1:
            import torch
            import torch.distributed as d
            if not d.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                d.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self._d, self._t = d, torch

    def barrier(self):
        if self._d:
            self._d.barrier()

    def max(self, v):
        return self._reduce(v, "MAX")

    def sum(self, v):
        return self._reduce(v, "SUM")

    def _reduce(self, v, op):
        if not self._d:
            return v
        t = self._t.tensor([float(v)], dtype=self._t.float64)
        self._d.all_reduce(t, op=getattr(self._d.ReduceOp, op))
        return float(t.item())

    def gather_object(self, obj):
        if not self._d:
            return [obj]
        out = [None] * self.world
        self._d.all_gather_object(out, obj)
        return out

    def close(self):
        if self._d and self._d.is_initialized():
            self._d.destroy_process_group()
