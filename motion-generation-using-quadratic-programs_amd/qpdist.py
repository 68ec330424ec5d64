"""qpdist — multi-GPU batch sharding for the batched solve.

The QPs of a batch are independent, so the path shards with no data-path collective: rank r
owns the contiguous block [r*B, (r+1)*B) of the global batch and generates or receives only
that block.  The only exchange is ONE gather of each batch's results (x, f, status) to rank 0,
which the reference's control loop would consume (src/mgqp.cpp:708-715 reads x and f of every
solve).  One process per GPU; backend "nccl" is RCCL on ROCm (xGMI peer links); "gloo" is used
by the CPU tests and by rehearsals with several ranks on one GPU.

Results travel packed, 68 B per QP at n = 7: the raw bits of x (n doubles), f (one double) and
status (one int32) as 2n + 3 int32 words per QP, so the gathered values are bit-exact.
"""
from __future__ import annotations

import numpy as np


def shard(rank: int, per_rank: int) -> tuple[int, int]:
    """Global QP index range owned by `rank` (`per_rank` QPs each)."""
    return rank * per_rank, (rank + 1) * per_rank


def packed_words(n: int) -> int:
    """int32 words per QP in the packed result record: x (2n), f (2), status (1)."""
    return 2 * n + 3


def pack_results_into(out, x, f, status):
    """Write (rows, n) float64 x, (B,) float64 f and (B,) int32 status into the (rows, 2n+3)
    int32 record `out` (torch tensors on one device, or numpy arrays).  Rows past B (the
    TILED64 padding of x) get f = status = 0.  Returns `out`."""
    rows, n = x.shape[0], x.shape[1]
    B = f.shape[0]
    try:
        import torch

        if isinstance(out, torch.Tensor):
            out[:, : 2 * n] = x.view(torch.int32).reshape(rows, 2 * n)
            out[:B, 2 * n: 2 * n + 2] = f.view(torch.int32).reshape(B, 2)
            out[:B, 2 * n + 2] = status
            if rows > B:
                out[B:, 2 * n:] = 0
            return out
    except ImportError:  # pragma: no cover
        pass
    out[:, : 2 * n] = np.ascontiguousarray(x, dtype=np.float64).view(np.int32).reshape(rows, 2 * n)
    out[:B, 2 * n: 2 * n + 2] = np.ascontiguousarray(f, dtype=np.float64).view(np.int32).reshape(B, 2)
    out[:B, 2 * n + 2] = status
    if rows > B:
        out[B:, 2 * n:] = 0
    return out


def pack_results(x, f, status):
    """numpy convenience: a new packed record of (x, f, status)."""
    x = np.asarray(x, dtype=np.float64)
    return pack_results_into(np.zeros((x.shape[0], packed_words(x.shape[1])), dtype=np.int32), x,
                             f, np.asarray(status, dtype=np.int32))


def unpack_results(parts, n: int, per_rank: int):
    """Concatenate the gathered per-rank records back into global (x, f, status) arrays."""
    xs, fs, ss = [], [], []
    for p in parts:
        a = np.ascontiguousarray(p.cpu().numpy() if hasattr(p, "cpu") else np.asarray(p))[:per_rank]
        xs.append(np.ascontiguousarray(a[:, : 2 * n]).view(np.float64))
        fs.append(np.ascontiguousarray(a[:, 2 * n: 2 * n + 2]).view(np.float64).reshape(-1))
        ss.append(a[:, 2 * n + 2].astype(np.int32))
    return np.concatenate(xs), np.concatenate(fs), np.concatenate(ss)


class ResultGather:
    """Per-batch gather of packed results to rank 0, overlapped with the next batches' solves.

    `slots` packed buffers rotate with the solve streams: submit(j, ...) packs slot j on the
    solve stream, and (RCCL) issues the gather on a communication stream that waits for the
    pack only, so the next solves keep running; before slot j is packed again, wait(j) makes
    the solve stream wait for its previous gather.  With gloo (CPU tests, ranks sharing one
    GPU) the records go through host memory.  Rank 0's received records per slot are
    `received(j)` (a list of `world` tensors)."""

    def __init__(self, dist, rank: int, world: int, slots: int, rows: int, n: int, device,
                 backend: str):
        import torch

        self.torch, self.dist = torch, dist
        self.rank, self.world, self.n = rank, world, n
        self.nccl = backend == "nccl"
        self.device = torch.device(device)
        pdev = self.device if self.nccl else torch.device("cpu")
        self.packed = [torch.empty((rows, packed_words(n)), dtype=torch.int32, device=pdev)
                       for _ in range(slots)]
        self.recv = [[torch.empty_like(self.packed[0]) for _ in range(world)] if rank == 0 else None
                     for _ in range(slots)]
        self.works = [None] * slots
        self.comm = torch.cuda.Stream(self.device) if self.nccl else None

    @property
    def bytes_per_rank(self) -> int:
        return int(self.packed[0].numel() * 4)

    def wait(self, j: int, stream=None):
        w = self.works[j]
        if w is None:
            return
        if self.nccl:
            with self.torch.cuda.stream(stream):
                w.wait()  # the current (solve) stream waits for the RCCL work
        else:
            w.wait()
        self.works[j] = None

    def submit(self, j: int, x, f, status, stream=None):
        torch = self.torch
        if self.nccl:
            with torch.cuda.stream(stream):
                pack_results_into(self.packed[j], x, f, status)
                done = torch.cuda.Event()
                done.record(stream)
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(done)
                self.works[j] = self.dist.gather(self.packed[j], self.recv[j], dst=0, async_op=True)
        else:
            if x.device.type == "cuda":
                with torch.cuda.stream(stream):
                    tmp = pack_results_into(torch.empty(self.packed[j].shape, dtype=torch.int32,
                                                        device=x.device), x, f, status)
                    self.packed[j].copy_(tmp.cpu())
            else:
                pack_results_into(self.packed[j], x, f, status)
            self.works[j] = self.dist.gather(self.packed[j], self.recv[j], dst=0, async_op=True)

    def drain(self):
        for j in range(len(self.works)):
            if self.works[j] is not None:
                self.works[j].wait()
                self.works[j] = None

    def received(self, j: int):
        return self.recv[j]

    def time_one(self, reps: int = 10) -> float:
        """Milliseconds of one slot's gather alone (blocking, after 2 untimed)."""
        import time

        torch = self.torch
        for _ in range(2):
            self.dist.gather(self.packed[0], self.recv[0], dst=0)
        if self.nccl:
            torch.cuda.synchronize(self.device)
        self.dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            self.dist.gather(self.packed[0], self.recv[0], dst=0)
        if self.nccl:
            torch.cuda.synchronize(self.device)
        return (time.perf_counter() - t0) * 1e3 / reps
