#!/usr/bin/env python3
"""Benchmark: batched Goldfarb–Idnani QP solves on MI355X (BASELINE.json metric).

One "step" = one batched solve (one launch of the gfx950 kernel through the C-ABI
qpgpu_solve_batched) over the rank's resident batch of synthetic QPs.  With N > 1 every rank
solves its own shard (weak scaling, no data-path collective: the QPs are independent);
--gather adds an RCCL gather of each step's results (x, f, status) to rank 0 on a separate
stream, overlapped with the following solves, for deployments that collect results centrally.  Inputs are
generated on the host from the counter-based generator (qpgpu.make_problems) and copied to HBM
before timing.

Steps are independent batches (one control period's QPs each), so they are pipelined: step k is
enqueued on HIP stream k mod S (--streams, default 3: GPU_MAX_HW_QUEUES is 4 and a fourth
stream measured sharing a hardware queue) with its own output buffers.  With 65 536
QPs a launch is exactly one wave per SIMD, so a single launch ends with most SIMDs idle behind
its slowest waves; the next step's waves fill them.  `value` is the pipelined whole-job
throughput; `roofline` uses the kernel's own duration from a separate serialized pass (HIP events
around each launch, one stream), which is what `rocprofv3 ... bench.py --streams 1` reports.

Default workload = BASELINE.json's metric config: 65 536 x (n=7, p=6, m=14) per GPU (weak
scaling: per-GPU work is fixed as N grows; C4's 1M QPs on 8 GPUs is --batch 131072 --gpus 8).

Single-GPU:  python bench.py [--steps K --warmup W]
Multi-GPU:   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "motion-generation-using-quadratic-programs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import qpdist  # noqa: E402
import qpgpu  # noqa: E402

METRIC = "QP solves/sec at n=7,p=6,m=14 batch=65536; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CONFIGS = {
    # name: (kind, n, p, m, default batch per GPU, description)
    "C1": ("general", 7, 6, 14, 65536, "C1/C4: 65536 x (n=7, p=6, m=14) general QPs per GPU"),
    "C2": ("box", 7, 0, 14, 65536, "C2: 65536 x (n=7, p=0, m=14) joint-limit box QPs per GPU"),
    "C3": ("general", 30, 6, 60, 65536, "C3: 65536 x (n=30, p=6, m=60) general QPs per GPU"),
    "mgqp": ("general", 14, 10, 28, 65536, "mgqp level-0 shape: 65536 x (n=14, p=10, m=28)"),
    "C5": ("general", 256, 0, 512, 4096, "C5: 4096 x (n=256, p=0, m=512) general QPs per GPU"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C1", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="QPs per GPU (default: config's)")
    ap.add_argument("--seed", type=int, default=2026)
    ap.add_argument("--family", default=None, choices=["lane", "subgroup", "wave"],
                    help="force a kernel family (default: the dispatcher's choice)")
    ap.add_argument("--layout", default="qp_major", choices=["qp_major", "tiled64"],
                    help="batch layout of the resident inputs (include/qpgpu.h)")
    ap.add_argument("--gather", action="store_true",
                    help="also gather every step's (x, f, status) to rank 0 over RCCL (N>1); off "
                         "by default: the QPs are independent, so the path has no exchange step")
    ap.add_argument("--streams", type=int, default=3,
                    help="HIP streams the steps are pipelined over (1 = serialized launches)")
    ap.add_argument("--kernel-reps", type=int, default=20,
                    help="serialized launches timed for the roofline's kernel duration")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def cpu_baseline(pr, seconds):
    """The oracle (CPU restatement, -O2, 1 thread) on the same resident batch, repeated until
    `seconds` of wall time: a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    oracle.lib()
    cap = 1000 + 100 * (pr.n + pr.p + pr.m)
    chunk = min(pr.batch, 8192)
    sub = pr.slice(0, chunk)
    done = 0
    t0 = time.perf_counter()
    while True:
        oracle.solve_batch(sub, max_steps=cap, threads=1)
        done += chunk
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    out = {"value": done / el, "unit": "QP solves/s", "cores": 1, "kind": "port",
           "sample": f"oracle/qp_oracle.c (-O2, 1 thread) re-solving the first {chunk} QPs of the "
                     f"same synthetic batch {done // chunk}x ({done} solves, {el:.1f} s)"}
    # the same restatement on the host's cores, one std::thread per core
    # over contiguous shards — capped at the CPU share a one-GPU box grants this job (16)
    threads = max(1, min(16, os.cpu_count() or 1))
    big = pr.slice(0, min(pr.batch, 8192 * 4))
    done_mt = 0
    t0 = time.perf_counter()
    while True:
        oracle.solve_batch(big, max_steps=cap, threads=threads)
        done_mt += big.batch
        el_mt = time.perf_counter() - t0
        if el_mt >= seconds / 2:
            break
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    out["multi_thread"] = {"value": done_mt / el_mt, "threads": threads, "cpu_model": model,
                           "sample": f"{big.batch} QPs per pass, {done_mt // big.batch} passes, "
                                     f"{el_mt:.1f} s"}
    out["cpu_model"] = model
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    dist = None
    # one rank per GPU; "nccl" is RCCL on ROCm.  QPGPU_DIST_BACKEND=gloo rehearses the N>1 flow
    # with several ranks on one GPU (results then travel through host memory).
    backend = os.environ.get("QPGPU_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    kind, n, p, m, bdef, desc = CONFIGS[args.config]
    B = args.batch or bdef
    b0, b1 = qpdist.shard(rank, B)
    pr = qpgpu.make_problems(kind, n, p, m, b0, b1, seed=args.seed)
    kname = qpgpu.kernel_name(n, p, m)
    if args.family:
        kname = {"lane": f"qp_lane[n={n},m={m}]", "subgroup": f"qp_small[n={n},m={m}]",
                 "wave": f"qp_wave[n={n},m={m}]"}[args.family]
    if not kname:
        sys.exit(f"no gfx950 kernel covers (n, p, m) = {(n, p, m)}")
    base = qpgpu.DeviceBatch(pr, dev, with_iters=False, layout=args.layout)
    S = max(1, args.streams)
    gather = world > 1 and args.gather

    def out_set():  # same resident inputs, private outputs
        b = qpgpu.DeviceBatch.__new__(qpgpu.DeviceBatch)
        b.__dict__.update(base.__dict__)
        b.x = torch.empty_like(base.x)
        b.f = torch.empty_like(base.f)
        b.status = torch.empty_like(base.status)
        return b

    bufs = [base] + [out_set() for _ in range(S - 1)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]  # non-default streams (no implicit sync)
    if gather:
        rows = base.x.shape[0]
        pdev = dev if backend == "nccl" else torch.device("cpu")
        packed = [torch.empty((rows, n + 2), dtype=torch.float64, device=pdev) for _ in range(S)]
        recv = [torch.empty((rows, n + 2), dtype=torch.float64, device=pdev) for _ in range(world)] if rank == 0 else None
        comm = torch.cuda.Stream(dev)
        works = [None] * S

    launch = [bufs[j].launcher(streams[j], family=args.family) for j in range(S)]

    def step(k):
        j = k % S
        db, cs = bufs[j], streams[j]
        if gather and works[j] is not None:
            # this stream's packed buffer is free once its gather finished: make stream cs
            # wait for it (Work.wait() syncs the *current* stream with an nccl work)
            with torch.cuda.stream(cs):
                works[j].wait()
            works[j] = None
        launch[j]()
        if gather:
            # pack (x, f, status) and gather to rank 0 on the comm stream, overlapping the
            # following steps' solves
            pk = packed[j]
            with torch.cuda.stream(cs):
                if backend == "nccl":
                    pk.copy_(qpdist.pack_results(db.x, db.f, db.status))
                    done = torch.cuda.Event()
                    done.record(cs)
                    with torch.cuda.stream(comm):
                        comm.wait_event(done)
                        works[j] = dist.gather(pk, recv if rank == 0 else None, dst=0, async_op=True)
                else:
                    pk.copy_(qpdist.pack_results(db.x, db.f, db.status).cpu())
                    works[j] = dist.gather(pk, recv if rank == 0 else None, dst=0, async_op=True)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    if gather:
        for w in works:
            if w is not None:
                w.wait()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # kernel-only duration for the roofline: serialized launches on one stream, HIP events
    # bracketing each launch on the stream it runs on (untimed for `value`)
    cs = streams[0]
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.kernel_reps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.kernel_reps)]
    for r in range(args.kernel_reps):
        starts[r].record(cs)
        launch[0]()
        ends[r].record(cs)
    torch.cuda.synchronize(dev)
    kern_ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in zip(starts, ends)]))
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    st = bufs[0].status.cpu().numpy()
    # every stream solved the same resident batch: identical outputs (guards the pipelining)
    consistent = all(torch.equal(bufs[0].f, b_.f) and torch.equal(bufs[0].x, b_.x) for b_ in bufs[1:])
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    total = B * world * args.steps
    value = total / elapsed
    bpq = qpgpu.algorithmic_bytes_per_qp(n, p, m)
    achieved = bpq * B / (kern_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    try:
        tj = json.load(open(args.traffic_json))
        key = f"{args.config}:{B}:{kname}"
        if key in tj:
            traffic = tj[key]["hbm_bytes_per_launch"]
            traffic_src = tj[key].get("source")
    except (OSError, ValueError):
        pass
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": desc, "kind": kind, "n": n, "p": p, "m": m, "batch_per_gpu": B,
                   "global_batch": B * world, "kernel": kname, "layout": args.layout,
                   "streams": S,
                   "parallelism": f"batch-sharded x{world}" + (", RCCL gather to rank 0 (overlapped)" if gather else ", no collective")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel_ms": kern_ms, "kernel_ms_source": "serialized launches, HIP events",
                     "algorithmic_bytes_per_qp": bpq,
                     "traffic_source": traffic_src},
        "status_ok_frac": float((st == qpgpu.QP_OK).mean()),
        "streams_outputs_identical": bool(consistent),
    }
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(pr, args.cpu_seconds)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
