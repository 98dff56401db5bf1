"""Multi-GPU sharding of a QP batch: one process per GPU, contiguous QP-id ranges, no data-path
collective. The counter-based generator keys every QP's inputs by its global id, so a QP's inputs and solution are
the same whatever the number of ranks; torch.distributed (gloo) is used only for barriers, the max-over-ranks time
and exchanging the 64-byte IPC handle of the result buffer. Results reach rank 0's GPU through ResultGather: each
rank writes its shard into rank 0's buffer with one device-to-device copy (xGMI peer write across GPUs, dmabuf IPC
mapping), so no collective and no reduction runs on the data path."""
import ctypes as C
import os
import sys


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
                # gloo prints "[Gloo] Rank r is connected to ..." on the process's stdout at rendezvous; bench.py's
                # stdout must carry only its JSON line, so fd 1 points at stderr while the group forms
                sys.stdout.flush()
                saved = os.dup(1)
                os.dup2(2, 1)
                try:
                    d.init_process_group("gloo", rank=self.rank, world_size=self.world)
                    d.barrier()  # every rank connected (and its message written) before stdout comes back
                finally:
                    sys.stdout.flush()
                    os.dup2(saved, 1)
                    os.close(saved)
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


class ResultGather:
    """Rank 0's gathered result buffer ([total_bytes] on rank 0's device), mapped into every rank's address space once
    (cmpc_ipc_export / cmpc_ipc_open, include/cmpc/cmpc.h) and reused for every gather. gather() copies this rank's
    shard to its byte offset with cmpc_gather_shard on `stream`, waits for it, then meets the other ranks at a
    barrier, after which rank 0's buffer holds every shard."""

    def __init__(self, dist, total_bytes):
        import cheeta_mpc as cm
        self.cm, self.dist, self.total = cm, dist, int(total_bytes)
        self.buf = None
        self.dst = C.c_void_p()
        self.mapped = False
        if dist.world == 1:
            self.buf = cm.DeviceArray((max(self.total, 1),), "uint8")
            self.dst = self.buf.ptr
        else:
            # every rank reaches each collective whatever fails locally (a rank that raised before a collective
            # would leave the others blocked in it): errors travel with the handle exchange and are raised after it
            hb, err = None, None
            if dist.rank == 0:
                try:
                    self.buf = cm.DeviceArray((max(self.total, 1),), "uint8")
                    self.dst = self.buf.ptr
                    h = cm.IpcHandle()
                    cm._chk(cm.lib().cmpc_ipc_export(self.buf.ptr, C.byref(h)), "cmpc_ipc_export")
                    hb = bytes(h.bytes)
                except Exception as e:  # noqa: BLE001 - re-raised below, after the exchange
                    err = e
            hb = dist.gather_object(hb)[0]
            if dist.rank != 0 and hb is None:
                err = RuntimeError("rank 0 could not export its result buffer")
            if dist.rank != 0 and err is None:
                try:
                    h = cm.IpcHandle()
                    C.memmove(C.addressof(h), hb, len(hb))
                    cm._chk(cm.lib().cmpc_ipc_open(C.byref(h), C.byref(self.dst)), "cmpc_ipc_open")
                    self.mapped = True
                except Exception as e:  # noqa: BLE001 - reported after the ranks agree
                    err = e
            # all ranks learn whether every rank is mapped; a failure anywhere fails the gather on every rank
            if dist.max(0.0 if err is None else 1.0) > 0.0:
                self.close()
                raise err if err is not None else RuntimeError("result gather unavailable on another rank")

    def gather(self, src_ptr, offset_bytes, nbytes, stream=None):
        cm = self.cm
        err = None
        try:
            if offset_bytes < 0 or offset_bytes + nbytes > self.total:
                raise ValueError("shard outside the gathered buffer")
            cm._chk(cm.lib().cmpc_gather_shard(self.dst, int(offset_bytes), src_ptr, int(nbytes), stream),
                    "cmpc_gather_shard")
            cm._hchk(cm.hip().hipStreamSynchronize(stream), "hipStreamSynchronize")
        except Exception as e:  # noqa: BLE001 - raised after the collective, so no rank is left waiting
            err = e
        if self.dist.max(0.0 if err is None else 1.0) > 0.0:  # the barrier, and every rank learns of a failure
            raise err if err is not None else RuntimeError("result gather failed on another rank")

    def host(self, dtype, shape):
        """Rank 0: the gathered buffer as a host array."""
        import numpy as np
        raw = self.buf.host()[: self.total]
        return raw.view(np.dtype(dtype)).reshape(shape)

    def close(self):
        if self.mapped:
            self.cm.lib().cmpc_ipc_close(self.dst)
            self.mapped = False
