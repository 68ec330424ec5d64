"""qpdist — multi-GPU batch sharding for the batched solve.

The QPs of a batch are independent, so the path shards with no data-path collective: rank r
owns the contiguous block [r*B, (r+1)*B) of the global batch (weak scaling, B per rank) and
generates or receives only that block.  The only exchange is the single gather of each step's
results (x, f, status) to rank 0, which the reference's control loop would consume
(src/mgqp.cpp:708-715 reads x and f of every solve).  One process per GPU; backend "nccl" is
RCCL on ROCm (xGMI peer links); "gloo" is used by the CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard(rank: int, per_rank: int) -> tuple[int, int]:
    """Global QP index range owned by `rank` (weak scaling: `per_rank` QPs each)."""
    return rank * per_rank, (rank + 1) * per_rank


def pack_results(x, f, status, rows: int | None = None):
    """(B, n) x, (B,) f, (B,) status -> one (rows, n+2) float64 tensor/array for a single gather.
    status is stored exactly (small integers are exact in binary64)."""
    try:
        import torch

        if isinstance(x, torch.Tensor):
            B, n = f.shape[0], x.shape[1]
            out = torch.zeros((rows or x.shape[0], n + 2), dtype=torch.float64, device=x.device)
            out[: x.shape[0], :n] = x
            out[:B, n] = f
            out[:B, n + 1] = status.to(torch.float64)
            return out
    except ImportError:  # pragma: no cover
        pass
    B, n = f.shape[0], x.shape[1]
    out = np.zeros((rows or x.shape[0], n + 2))
    out[: x.shape[0], :n] = x
    out[:B, n] = f
    out[:B, n + 1] = status
    return out


def unpack_results(parts, n: int, per_rank: int):
    """Concatenate the gathered per-rank blocks back into global (x, f, status) arrays."""
    xs, fs, ss = [], [], []
    for p in parts:
        a = p.cpu().numpy() if hasattr(p, "cpu") else np.asarray(p)
        xs.append(a[:per_rank, :n])
        fs.append(a[:per_rank, n])
        ss.append(a[:per_rank, n + 1].astype(np.int32))
    return np.concatenate(xs), np.concatenate(fs), np.concatenate(ss)


def gather_to_rank0(dist, packed, rank: int, world: int, async_op: bool = False):
    """One gather of every rank's packed results to rank 0 (RCCL gather over xGMI with the
    nccl backend).  Returns (work, recv_list) — recv_list is None except on rank 0."""
    import torch

    recv = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    work = dist.gather(packed, recv, dst=0, async_op=async_op)
    return work, recv
