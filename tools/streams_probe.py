#!/usr/bin/env python3
"""Probe: C1 batched solves issued round-robin on S HIP streams (independent output buffers), so
one launch's slowest-wave tail overlaps the next launch's head.  Prints ms per launch for each S."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))
import torch  # noqa: E402

import qpgpu  # noqa: E402


def main():
    pr = qpgpu.make_problems("general", 7, 6, 14, 0, 65536, seed=2026)
    dev = torch.device("cuda", 0)
    base = qpgpu.DeviceBatch(pr, dev, with_iters=False)
    K = 200
    for S in (1, 2, 3, 4, 6, 8):
        bufs = []
        for _ in range(S):
            b = qpgpu.DeviceBatch.__new__(qpgpu.DeviceBatch)
            b.__dict__.update(base.__dict__)
            b.x, b.f, b.status = torch.empty_like(base.x), torch.empty_like(base.f), torch.empty_like(base.status)
            bufs.append(b)
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        L = [bufs[j].launcher(streams[j]) for j in range(S)]
        for k in range(20):
            L[k % S]()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(K):
            L[k % S]()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        print(f"streams={S}: {el / K * 1e3:.4f} ms per launch, {65536 * K / el:.3e} solves/s", flush=True)


if __name__ == "__main__":
    main()
