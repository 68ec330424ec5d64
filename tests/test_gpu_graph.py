"""hipGraph capture of the batched solve (include/qpgpu.h: qpgpu_solve_batched only enqueues work
on its stream and never synchronises, so it can be captured; kernels that use a device workspace
— n > 64, and the generic kernel — need one call on the capturing stream first, which allocates
the workspace outside the capture).  A captured solve replayed on new inputs copied into the
captured buffers must give exactly what a direct solve of those inputs gives."""
import numpy as np
import pytest

import qpgpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,n,p,m,B,fast,family", [
    ("general", 7, 6, 14, 4096, True, None),      # qp_lane_fast (C1)
    ("general", 7, 6, 14, 4096, False, None),     # qp_lane (bitwise)
    ("general", 14, 10, 28, 2048, True, None),    # qp_wave_fast (mgqp level)
    ("general", 100, 5, 200, 8, False, None),     # MFMA panel setup + workspace loop (two kernels)
    ("general", 20, 3, 40, 64, False, "generic"),  # generic workspace kernel
])
def test_captured_solve_replays_exactly(gpu, kind, n, p, m, B, fast, family):
    import torch

    dev = torch.device("cuda", 0)
    pr1 = qpgpu.make_problems(kind, n, p, m, 0, B, seed=100 + n)
    pr2 = qpgpu.make_problems(kind, n, p, m, B, 2 * B, seed=100 + n)  # other QPs, same shape
    db = qpgpu.DeviceBatch(pr1, dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        db.solve(stream=s, fast=fast, family=family)  # warm-up on the capturing stream
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        db.solve(stream=s, fast=fast, family=family)
    # replay on pr2's inputs: copy them into the captured input tensors
    for name, a in zip(("G", "g0", "CE", "ce0", "CI", "ci0"), pr2.arrays()):
        getattr(db, name).copy_(torch.from_numpy(np.ascontiguousarray(a)).reshape(getattr(db, name).shape))
    g.replay()
    torch.cuda.synchronize()
    xg, fg, sg, ig = db.results()
    ref = qpgpu.DeviceBatch(pr2, dev)
    ref.solve(fast=fast, family=family)
    torch.cuda.synchronize()
    xr, fr, sr, ir = ref.results()
    assert np.array_equal(sg, sr) and np.array_equal(ig, ir)
    assert np.array_equal(fg.view(np.uint64), fr.view(np.uint64))
    ok = sr != qpgpu.QP_NOT_POSITIVE_DEFINITE
    assert np.array_equal(xg[ok].view(np.uint64), xr[ok].view(np.uint64))
    # and once more with the first inputs: the graph is reusable
    for name, a in zip(("G", "g0", "CE", "ce0", "CI", "ci0"), pr1.arrays()):
        getattr(db, name).copy_(torch.from_numpy(np.ascontiguousarray(a)).reshape(getattr(db, name).shape))
    g.replay()
    torch.cuda.synchronize()
    x1, f1, s1, _ = db.results()
    d1 = qpgpu.DeviceBatch(pr1, dev)
    d1.solve(fast=fast, family=family)
    torch.cuda.synchronize()
    x1r, f1r, s1r, _ = d1.results()
    assert np.array_equal(s1, s1r) and np.array_equal(f1.view(np.uint64), f1r.view(np.uint64))
