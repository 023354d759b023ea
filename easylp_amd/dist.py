"""Multi-rank plumbing for the column-sharded solve.

Production: one process per GPU over RCCL -- rank 0 creates the 128-byte
RCCL unique id (elp_comm_unique_id), `share_unique_id` ships it with
torch.distributed, every rank calls Problem.comm_init(id, world, rank).

Tests: `TorchDistTransport` implements the three host-transport callbacks of
elp_comm_init_host (all-gather, all-reduce f64-sum / i32-max, broadcast) with
torch.distributed on CPU tensors (gloo), so several ranks can share one GPU
(RCCL refuses two ranks on one device) and the sharded kernels still run.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ._lib import ALLGATHER_FN, ALLREDUCE_FN, BCAST_FN


def _view(addr: int, nbytes: int) -> torch.Tensor:
    buf = (ctypes.c_uint8 * nbytes).from_address(addr)
    return torch.frombuffer(buf, dtype=torch.uint8)


def share_unique_id(lib, rank: int) -> bytes:
    """Rank 0 makes the RCCL unique id; every rank returns the same 128 bytes."""
    uid = ctypes.create_string_buffer(128)
    if rank == 0:
        rc = lib.elp_comm_unique_id(uid)
        if rc < 0:
            raise RuntimeError("elp_comm_unique_id failed: " + lib.elp_last_error().decode())
    obj = [uid.raw if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


class TorchDistTransport:
    """Host transport over torch.distributed (any backend with CPU tensors)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.errors = 0
        # keep the ctypes thunks alive as long as the transport
        self.c_allgather = ALLGATHER_FN(self._allgather)
        self.c_allreduce = ALLREDUCE_FN(self._allreduce)
        self.c_bcast = BCAST_FN(self._bcast)

    # -- python-level primitives (also used directly by the CPU tests) --
    def allgather_bytes(self, send: bytes) -> bytes:
        t = torch.frombuffer(bytearray(send), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return b"".join(o.numpy().tobytes() for o in out)

    def allreduce_f64_sum(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def allreduce_i32_max(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)

    # -- C callbacks: pointers into host staging buffers owned by the library --
    def _allgather(self, send, recv, nbytes, user):
        try:
            data = self.allgather_bytes(bytes(_view(send, nbytes).numpy()))
            ctypes.memmove(recv, data, len(data))
            return 0
        except Exception:  # never let an exception cross the C boundary
            self.errors += 1
            return 1

    def _allreduce(self, buf, count, dtype, user):
        try:
            if dtype == 0:
                t = torch.frombuffer((ctypes.c_double * count).from_address(buf), dtype=torch.float64)
                self.allreduce_f64_sum(t)
            else:
                t = torch.frombuffer((ctypes.c_int32 * count).from_address(buf), dtype=torch.int32)
                self.allreduce_i32_max(t)
            return 0
        except Exception:
            self.errors += 1
            return 1

    def _bcast(self, buf, nbytes, root, user):
        try:
            t = _view(buf, nbytes)
            dist.broadcast(t, src=int(root), group=self.group)
            return 0
        except Exception:
            self.errors += 1
            return 1
