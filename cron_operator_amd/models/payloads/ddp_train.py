"""Example scheduled payload: data-parallel training over RCCL on MI355X GPUs.

Workload data for the ``examples/mi355x`` Cron templates (a nightly PyTorchJob
on one 8x MI355X node).  It is launched by the training-operator (or this
repo's fake training-operator in real mode) with the standard PyTorchJob env:
``MASTER_ADDR``/``MASTER_PORT``/``WORLD_SIZE``/``RANK`` (one process per
replica) -- or by ``torchrun --nproc-per-node 8`` inside a single replica, which
sets ``LOCAL_RANK`` too.

One process per GPU, ``torch.distributed`` with backend ``nccl`` (RCCL on ROCm;
xGMI between the 8 GPUs of a node), ``DistributedDataParallel`` with a bucket
size sized for point-to-point xGMI rings (``--bucket-mb``, default 100 MB:
fewer, larger all-reduces), bf16 autocast, synthetic data.  Falls back to
``gloo`` on CPU so the same file runs in CPU tests.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _allreduce_busbw(torch, dist, dev, mb: int, world: int, iters: int = 10, warmup: int = 3) -> dict:
    """Time ``iters`` all-reduces of one ``mb``-MB bf16 buffer -- the size class of a DDP gradient
    bucket -- and return the ring bus bandwidth ``2(n-1)/n * bytes / t`` (the per-link figure to
    hold against xGMI's ~153 GB/s per link), the max over ranks of each rank's mean time."""
    n = max(1, mb * 1024 * 1024 // 2)
    buf = torch.ones(n, dtype=torch.bfloat16, device=dev)
    for _ in range(warmup):
        dist.all_reduce(buf)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    t = float(dt.item())
    nbytes = n * 2
    return {"mb": mb, "iters": iters, "ms": round(t * 1000, 3),
            "algbw_gbs": round(nbytes / t / 1e9, 2),
            "busbw_gbs": round(2 * (world - 1) / world * nbytes / t / 1e9, 2)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (kernel selection, RCCL setup); default 3 on GPUs, 0 on CPU")
    ap.add_argument("--batch", type=int, default=32, help="per-rank batch")
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--bucket-mb", type=int, default=100)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--allreduce-mb", type=int, default=0,
                    help="after training, time an all-reduce of this many MB of bf16 and report its bus "
                         "bandwidth (0: skip)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist

    use_gpu = torch.cuda.is_available() and not a.cpu
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank % max(1, torch.cuda.device_count() if use_gpu else 1))))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    dev = torch.device(f"cuda:{local}" if use_gpu else "cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    dist.init_process_group("nccl" if use_gpu else "gloo", rank=rank, world_size=world)

    torch.manual_seed(1234)
    blocks = []
    for _ in range(a.layers):
        blocks += [torch.nn.Linear(a.hidden, 4 * a.hidden), torch.nn.GELU(), torch.nn.Linear(4 * a.hidden, a.hidden)]
    model = torch.nn.Sequential(*blocks).to(dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local] if use_gpu else None,
                                                    bucket_cap_mb=a.bucket_mb, gradient_as_bucket_view=True)
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-4, fused=use_gpu)
    gen = torch.Generator(device="cpu").manual_seed(rank)
    x = torch.randn(a.batch, a.hidden, generator=gen).to(dev)
    y = torch.randn(a.batch, a.hidden, generator=gen).to(dev)
    def step():
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=use_gpu):
            out = torch.nn.functional.mse_loss(ddp(x).float(), y)
        opt.zero_grad(set_to_none=True)
        out.backward()
        opt.step()
        return out

    loss = None
    for _ in range(a.warmup if a.warmup is not None else (3 if use_gpu else 0)):
        loss = step()
    if use_gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    if use_gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # parameters must be identical on every rank after DDP steps
    flat = torch.cat([p.detach().float().reshape(-1)[:64] for p in model.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    in_sync = bool(torch.allclose(flat, ref))
    # which physical device each rank trained on (PCI bus id on GPUs): ranks must not share one
    if use_gpu:
        props = torch.cuda.get_device_properties(dev)
        ident = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    else:
        ident = f"cpu:{rank}"
    devices = [None] * world
    dist.all_gather_object(devices, ident)
    allreduce = None
    if a.allreduce_mb > 0:  # one rank has no peer to exchange with: its "all-reduce" moves nothing
        allreduce = (_allreduce_busbw(torch, dist, dev, a.allreduce_mb, world) if world > 1
                     else {"mb": a.allreduce_mb, "skipped": "world 1: no peers"})
    if rank == 0:
        print("DDP_OK " if in_sync else "DDP_FAIL ", json.dumps({
            "world": world, "backend": dist.get_backend(), "device": str(dev), "devices": devices,
            "visible_devices": torch.cuda.device_count() if use_gpu else 0, "loss": float(loss.detach()),
            "steps_per_s": a.steps / dt, "samples_per_s": a.steps * a.batch * world / dt,
            "allreduce": allreduce}), flush=True)
    # every rank leaves its last collective before any rank tears its connections down: a gloo
    # peer that closes while another still reads from it can abort that rank (SIGABRT) at exit
    dist.barrier()
    dist.destroy_process_group()
    return 0 if in_sync else 1


if __name__ == "__main__":
    sys.exit(main())
