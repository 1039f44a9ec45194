"""Smoke payload a scheduled PyTorchJob runs on an MI355X: one tiny training step.

This is *workload data*, not operator code: the example/smoke Cron templates
put ``python -m cron_operator_amd.models.payloads.train_smoke`` in the Master
container, and the fake training-operator (real mode) runs it as the replica
process.  It does one forward + backward + optimizer step of a small MLP in
bf16 on ``cuda:0`` (the ROCm HIP device under PyTorch-ROCm), checks the
gradients against an fp32 CPU reference of the same step, and prints
``SMOKE_OK`` with the device name.  Exit code 0 marks the job Succeeded.

``--device cpu`` runs the same step on the CPU (used by CPU-only tests).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default=os.environ.get("SMOKE_DEVICE", "cuda:0"))
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)

    t0 = time.perf_counter()
    import torch

    if a.device.startswith("cuda") and not torch.cuda.is_available():
        print("SMOKE_FAIL no GPU visible to PyTorch", flush=True)
        return 2
    torch.manual_seed(a.seed)
    dev = torch.device(a.device)
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32

    def build():
        torch.manual_seed(a.seed)
        return torch.nn.Sequential(torch.nn.Linear(a.hidden, 4 * a.hidden), torch.nn.GELU(),
                                   torch.nn.Linear(4 * a.hidden, a.hidden), torch.nn.LayerNorm(a.hidden),
                                   torch.nn.Linear(a.hidden, 10))

    gen = torch.Generator().manual_seed(a.seed + 1)
    x = torch.randn(a.batch, a.hidden, generator=gen)
    y = torch.randint(0, 10, (a.batch,), generator=gen)

    model = build().to(dev, dtype)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    loss = torch.nn.functional.cross_entropy(model(x.to(dev, dtype)).float(), y.to(dev))
    loss.backward()
    grad0 = model[0].weight.grad.float().cpu()
    opt.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()

    # fp32 CPU reference of the same step
    ref = build().float()
    ref_loss = torch.nn.functional.cross_entropy(ref(x), y)
    ref_loss.backward()
    gref = ref[0].weight.grad
    rel = float((grad0 - gref).norm() / (gref.norm() + 1e-12))
    ok = bool(torch.isfinite(loss).item()) and abs(float(loss) - float(ref_loss)) < 0.05 and rel < 0.05
    info = {"device": str(dev), "name": torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu",
            "hip": getattr(torch.version, "hip", None), "loss": float(loss), "ref_loss": float(ref_loss),
            "grad_rel_err": rel, "seconds": round(time.perf_counter() - t0, 3),
            "job": os.environ.get("KUBEFLOW_JOB_NAME", ""), "rank": os.environ.get("RANK", "0")}
    print(("SMOKE_OK " if ok else "SMOKE_FAIL ") + json.dumps(info), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
