"""The RCCL branch of the multi-GPU path on a real device: a world-size-1
"nccl" process group (RCCL on ROCm) bound to cuda:0 with device_id, as bench.py's ranks create
it, and qpdist.ResultGather driven through its nccl code path — packing on the solve stream, the
communication stream waiting on the pack event, the asynchronous gather, and the solve stream
waiting on the gather's work object before the slot is packed again.  The record rank 0
receives must be the packed results bit for bit, and unpack to the solve's x, f, status.

(world size > 1 is exercised with gloo on CPU in tests/test_multirank_cpu.py; RCCL with several
ranks needs one GPU per rank, which only the driver's multi-GPU runs have.)"""
import socket

import numpy as np
import pytest

import qpdist
import qpgpu

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_result_gather_world1(gpu):
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        n, B, S = 7, 4096, 2
        prs = [qpgpu.make_problems("general", n, 6, 14, k * B, (k + 1) * B, seed=2026) for k in range(3)]
        dbs = [qpgpu.DeviceBatch(p, dev, with_iters=False) for p in prs]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        gat = qpdist.ResultGather(dist, 0, 1, S, B, n, dev, "nccl")
        assert gat.nccl and gat.comm is not None
        # three batches over two slots: slot 0 is reused, so its second pack must wait for the
        # first gather (wait() on the solve stream)
        for k, db in enumerate(dbs):
            j = k % S
            cs = streams[j]
            gat.wait(j, cs)
            db.solve(stream=cs, fast=True)
            gat.submit(j, db.x, db.f, db.status, stream=cs)
            if k == 0:
                gat.wait(0, cs)
                torch.cuda.synchronize(dev)
                got0 = gat.received(0)[0].clone()
        gat.drain()
        torch.cuda.synchronize(dev)
        for j, k in ((0, 2), (1, 1)):
            rec = gat.received(j)
            assert len(rec) == 1 and rec[0].device.type == "cuda"
            assert torch.equal(rec[0], gat.packed[j]), f"slot {j}: received != packed"
            x, f, st = qpdist.unpack_results(rec, n, B)
            xr, fr, sr, _ = dbs[k].results()
            assert np.array_equal(x.view(np.uint64), xr.view(np.uint64))
            assert np.array_equal(f.view(np.uint64), fr.view(np.uint64))
            assert np.array_equal(st, sr)
        # the first batch's record, taken before slot 0 was reused
        x0, f0, s0 = qpdist.unpack_results([got0], n, B)
        solo = qpgpu.DeviceBatch(prs[0], dev, with_iters=False)
        solo.solve(fast=True)
        torch.cuda.synchronize(dev)
        xs, fs, ss, _ = solo.results()
        assert np.array_equal(x0.view(np.uint64), xs.view(np.uint64)) and np.array_equal(s0, ss)
        assert gat.time_one(reps=3) > 0.0
    finally:
        dist.destroy_process_group()
