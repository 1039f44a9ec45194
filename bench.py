#!/usr/bin/env python3
"""Headline benchmark: reconcile throughput + tick->create latency @ 1000 Cron CRs.

BASELINE.json names the metric "reconciles/sec + p50 schedule->create latency
@1000 Cron CRs" on the config "1000 Cron CRs at ``* * * * *``, historyLimit=10
-- reconcile-throughput + GC stress".  This runs exactly that (see
``cron_operator_amd/bench/harness.py`` for the step definition): every timed
step is one schedule tick in virtual time in which all 1000 Crons move their
finished job into history, garbage-collect the overflow, create the tick's
PyTorchJob and update status -- against a fake Kubernetes apiserver running in
its own process, over HTTP + watch streams.  Synthetic objects, no cluster.

Each rank runs the operator as ``--shards`` (default 3; fewer when the CPUs available
to the job cannot give each rank a core per shard plus one for its apiserver) shard processes of the
operator's horizontal sharding feature: the reference's Go controller spreads its 10 reconcile
workers over all cores as goroutines, and sharding is how this asyncio operator uses more than
one core.  ``--shards 1`` keeps a single operator process.  ``--shard-routing labels`` (default)
has each shard watch only its own Crons and children (``kubedl.io/shard`` labels, assigned by
the shards during setup); ``hash`` has every shard watch everything.

The fake cluster (``--fixture``).  A real apiserver serves from many cores; the fake one is one
server thread, and one of them saturates under 3 shards (0.87-0.93 busy in round 6: the number
then measured the fixture as much as the operator).  So by default (``partitioned``) each shard
gets a fake apiserver process of its own, holding the Crons that hash to that shard and their
jobs -- exactly what that shard watches and writes under label routing -- and the headline
measures the shards (busiest partition ~0.4-0.6 busy on the box).  It needs two CPUs per shard
plus one per rank (3 shards from 7 CPUs per rank, 2 from 5); below 5 the headline falls back to
``shared``: every shard against one fake apiserver, the rounds 1-5 layout.
``shared_fixture_*`` (or ``partitioned_*`` when the headline is shared) is the same shards
against the other layout, in this same invocation after the timed run (``--other-fixture
none`` skips it); ``config.fixture`` says which one the headline used.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it runs under ``torch.distributed.run`` with one rank per GPU (without a launcher,
``--gpus N`` spawns the N rank processes itself).  The operator is
pure control plane, so ranks do not use the GPU: each
rank is one operator deployment (its shards, its own fake apiserver processes and 1000
Crons: weak scaling) and rank 0 reports the whole-job aggregate.  Ranks synchronise with
gloo barriers; there is no device work to ``torch.cuda.synchronize()``.

``single_process_*``: the chart ships ONE operator process (``sharding.count: 1``,
``processes: 1``); it runs in the same invocation on the same Crons, after the timed run
(``--single-process none`` skips it).  ``operator_cpu_ms_per_fire`` and ``apiserver_busy_frac``
(and their ``single_process_`` / ``shared_fixture_`` twins) say which side bounds each number:
near 1.0 busy, the fake apiserver does (``apiserver_busy_frac`` is the busiest fake apiserver's
CPU s per wall s; ``apiserver_cpu_us_per_fire`` counts all of them).  Since round 6 the fixture
is native C++ (``--apiserver-impl native``, ``ops/csrc/apiserverd.cpp``); the Python fixture of
rounds 1-5 ran 0.94 busy at 3 shards and 0.86 for one process (``--apiserver-impl python``).

``deployment_*``: a real cluster is latency-bound, not CPU-bound: TLS on every connection and an
etcd quorum write behind every mutation.  ``deployment_value`` / ``deployment_baseline_value`` are
both algorithms in that shape (one process each, TLS + the harness's ``etcd`` latency model, whose
``list_per_object`` charges the namespace scan a real apiserver does for a label-selected LIST), run
in this same invocation after the timed run; ``vs_baseline_deployment`` is their ratio
(``--deployment none`` skips them).

Job lifecycle.  The headline (and its single-process and reference runs) keeps the rounds 1-4
step: each job of the previous tick is marked Succeeded in one write (``--lifecycle instant``).
The fake apiserver applies those writes a few per loop turn, between the turns serving the
operator (``--completion-writes interleaved``; ``batch`` applies all of them in one call, as in
rounds 1-5); their fixture CPU is inside the timed region either way.
The deployment-shaped pair runs the realistic sequence (``--deployment-lifecycle realistic``):
the training-operator's ``Created``, one ``replicaStatuses`` write per pod, ``Running``, then
``Succeeded``, each absorbed by the operator before the next.  Every such write changes the job's
resourceVersion, which the reference folds into ``status.active`` (``cron_controller.go:284-304``):
it pays a reconcile, a live LIST and a status PATCH per write, this operator nothing
(``deployment_api_requests_per_fire``).  The harness's own write calls are not timed; the
operator's absorption of each write is.

``payload_ddp``: last of all, untimed, when the node has a GPU per rank, rank 0 runs the
payload the operator schedules (``models/payloads/ddp_train.py``: DDP over RCCL, one process
per GPU) as a time-limited child job on those GPUs and reports whether its ranks stayed in
sync and a 256 MB all-reduce's bus bandwidth -- so the driver's N-GPU runs also exercise
RCCL over xGMI at N ranks (``--payload-probe none`` skips it).

``vs_baseline``: the reference publishes no numbers, so the denominator
is the reference *algorithm* (``--mode reference``: live LIST per reconcile, status
churn, no event filtering) run by this same invocation on the same Crons, after the
timed run.  ``operator_cpu_ms_per_fire`` and ``apiserver_busy_frac`` show how much of
the headline is the operator and how much the fake apiserver fixture.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# BASELINE.md row "Reference algorithm, measured in this harness" (cron-reconciles/s @1000 Crons,
# `--mode reference`, MI355X box, r1i: profiles/shard_sweep_mi355x_box_r1i.json).  Only used with
# `--baseline recorded`; by default the denominator is measured in the same invocation (below).
RECORDED_BASELINE_VALUE = 80.72


def _spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script and exit with the
    worst exit code.  The ranks rendezvous through a file (no port to race other jobs for); a
    rank that fails ends the others instead of leaving them waiting at a barrier.  Nothing here
    touches the GPU, so child processes are started, never exec'd.  Only rank 0 prints the
    JSON line."""
    import shutil
    import subprocess
    import tempfile

    rdzv_dir = tempfile.mkdtemp(prefix="bench-rdzv-")
    rdzv = os.path.join(rdzv_dir, "store")  # created by the first rank's FileStore
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", BENCH_RDZV_FILE=rdzv)
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        rcs = [None] * n
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                rcs = [p.wait() if rc is None else rc for p, rc in zip(procs, rcs)]
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        shutil.rmtree(rdzv_dir, ignore_errors=True)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def _payload_probe(world: int, timeout_s: float, cpu: bool = False, allreduce_mb: int = 256,
                   steps: int = 20) -> dict:
    """Untimed, after everything else: the scheduled workload's own data path on this node.

    The operator never touches the GPU; what it schedules does (``examples/mi355x``: a nightly
    PyTorchJob of one process per GPU, DDP over RCCL/xGMI).  When this node has a GPU per rank,
    rank 0 launches that payload (``models/payloads/ddp_train.py``) as a CHILD
    ``torch.distributed.run`` with ``world`` processes, one per GPU, in its own session and under a
    hard time limit, and reports its result: ranks in sync, the distinct devices used, and the
    bus bandwidth of a 256 MB bf16 all-reduce.  A failure or timeout is reported, never raised:
    it must not cost the headline line."""
    import signal
    import socket
    import subprocess

    if not cpu:
        if not os.path.exists("/dev/kfd"):
            return {"skipped": "no GPU on this node"}
        try:
            import torch

            visible = torch.cuda.device_count()  # counting does not initialise the GPU in this process
        except Exception as e:  # noqa: BLE001
            return {"skipped": f"torch: {type(e).__name__}"}
        if visible < world:
            return {"skipped": f"{visible} visible GPUs < {world} ranks"}
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "BENCH_RDZV_FILE")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           "-m", "cron_operator_amd.models.payloads.ddp_train", "--steps", str(steps),
           "--allreduce-mb", str(allreduce_mb)] + (["--cpu", "--hidden", "64", "--batch", "4"] if cpu else [])
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"error": f"timed out after {timeout_s:.0f} s", "world": world}
    res: dict = {"rc": p.returncode, "wall_s": round(time.perf_counter() - t0, 1)}
    for line in out.splitlines():
        if line.startswith(("DDP_OK ", "DDP_FAIL ")):
            tag, _, body = line.partition(" ")
            try:
                info = json.loads(body)
            except ValueError:
                break
            res.update({"ok": tag == "DDP_OK" and p.returncode == 0, "world": info.get("world"),
                        "backend": info.get("backend"), "distinct_devices": len(set(info.get("devices") or [])),
                        "ddp_steps_per_s": round(info.get("steps_per_s", 0.0), 2),
                        "allreduce": info.get("allreduce")})
            return res
    res["error"] = (out.strip().splitlines() or ["no output"])[-1][:300]
    return res


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return None, 0, 1
    from datetime import timedelta

    import torch.distributed as dist  # only multi-rank runs pay for importing torch

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    rdzv = os.environ.get("BENCH_RDZV_FILE")
    # a rank that never arrives fails the others after this long instead of hanging them
    timeout = timedelta(seconds=float(os.environ.get("BENCH_RDZV_TIMEOUT_S", "900")))
    if rdzv:  # ranks spawned by _spawn_ranks
        dist.init_process_group("gloo", init_method=f"file://{rdzv}", rank=int(os.environ["RANK"]),
                                world_size=ws, timeout=timeout)
    else:  # torch.distributed.run: env:// (MASTER_ADDR / MASTER_PORT)
        dist.init_process_group("gloo", timeout=timeout)
    return dist, dist.get_rank(), dist.get_world_size()


def _progress(rank: int, msg: str) -> None:
    """One progress line on stderr (stdout carries only the JSON line): a long invocation
    is never silent for minutes."""
    if rank == 0:
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def _barrier(dist) -> None:
    if dist is not None:
        dist.barrier()


def _sync_device() -> None:
    """No kernels are launched by the operator; synchronise only if a device was touched."""
    if "torch" in sys.modules:
        import torch

        if torch.cuda.is_initialized():
            torch.cuda.synchronize()


def _latency_ceiling(allr, workers: int, crons: int, history_limit: int, model: dict):
    """Fires/s (all ranks) the reference algorithm could reach if its only cost were the
    latency model's wait per request: ``workers`` reconciles at a time, each awaiting its
    requests one after another (``cron_controller.go:90-239``).  A label-selected LIST also
    pays ``list_per_object`` per object in the namespace (``crons x (historyLimit + 1)`` jobs)."""
    total = 0.0
    for r in allr:
        by_verb = r.get("dep_ref_by_verb") or {}
        fires = r.get("dep_ref_fires") or 0
        if not fires:
            return None
        wait = sum(n * model.get(v, 0.0) for v, n in by_verb.items())
        wait += by_verb.get("list", 0) * model.get("list_per_object", 0.0) * crons * (history_limit + 1)
        if wait <= 0:
            return None
        total += workers * fires / wait
    return round(total, 2)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[1])
    ap.add_argument("--gpus", type=int, default=1)
    # no flags: 10 ticks after 5 of warm-up (on the box the first two or three ticks of fresh
    # processes run 2.5-3x slower than the rest: `r6w_startup_ticks` in
    # profiles/bench_driver_shape_mi355x_box_r6g.json)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--history-limit", type=int, default=10)
    ap.add_argument("--workers", type=int, default=10, help="--max-concurrent-reconciles")
    ap.add_argument("--qps", type=float, default=-1.0, help="client QPS (-1: unthrottled)")
    ap.add_argument("--burst", type=int, default=50)
    ap.add_argument("--max-inflight", type=int, default=128,
                    help="client cap on concurrent API requests (--max-inflight-requests; 0: unlimited)")
    ap.add_argument("--no-defer", action="store_true",
                    help="A/B: reconcile writes on the worker (ReconcilerOptions.defer_status_write=False)")
    ap.add_argument("--transport", choices=["http", "memory"], default="http")
    ap.add_argument("--mode", choices=["optimized", "reference"], default="optimized")
    ap.add_argument("--shards", type=int, default=0,
                    help="operator shards per rank (--shard-count): the reference's controller spreads its 10 "
                         "workers over every core as goroutines; this asyncio operator uses cores by sharding. "
                         "0 (default): 3, or fewer when the CPUs available to the job cannot give every rank "
                         "one core per shard plus one for its apiserver")
    ap.add_argument("--shard-routing", choices=["hash", "labels"], default="labels",
                    help="how shards split the watch traffic (controller/sharding.py)")
    ap.add_argument("--apiserver-latency", choices=["none", "etcd"], default="none",
                    help="server-side per-verb latency model of the fake apiserver (harness LATENCY_PROFILES)")
    ap.add_argument("--apiserver-impl", choices=["native", "python"], default="native",
                    help="the fake apiserver fixture: native (C++ _apiserverd, off the critical path) or python "
                         "(apiserver/server.py + http.py, the rounds 1-5 fixture; A/B)")
    ap.add_argument("--tls", action="store_true",
                    help="the fake apiserver serves HTTPS and the operator verifies it against its CA, as "
                         "against a real cluster (every operator connection is TLS)")
    ap.add_argument("--baseline", choices=["measure", "recorded", "none"], default="measure",
                    help="vs_baseline denominator: 'measure' runs the reference algorithm (--mode reference, "
                         "one operator process, same Crons) in this same invocation after the timed run; "
                         "'recorded' divides by the BASELINE.md figure")
    ap.add_argument("--single-process", choices=["measure", "none"], default="measure",
                    help="also run the shipped default -- ONE operator process (the chart's sharding.count=1, "
                         "processes=1) -- on the same 1000 Crons in this invocation, outside the headline's timed "
                         "region, and report it as single_process_*: operator-bound, so it measures the product "
                         "rather than the fake apiserver")
    ap.add_argument("--fixture", choices=["partitioned", "shared"], default="partitioned",
                    help="the headline's fake apiserver with more than one shard: 'partitioned' (default) -- one "
                         "apiserver process per shard, holding the Crons that hash to it and their jobs, so no "
                         "single-threaded fixture bounds the shards (needs 2 CPUs per shard + 1 per rank; 'shared' "
                         "otherwise) -- or 'shared', every shard against one apiserver process (rounds 1-5)")
    ap.add_argument("--other-fixture", choices=["measure", "none"], default="measure",
                    help="also run the headline's shards against the other fixture layout, outside the "
                         "headline's timed region: shared_fixture_* (or partitioned_*) keys")
    ap.add_argument("--single-steps", type=int, default=10)
    ap.add_argument("--single-warmup", type=int, default=3)
    ap.add_argument("--deployment", choices=["measure", "none"], default="measure",
                    help="also run both algorithms deployment-shaped (1 process, TLS + etcd latency model) in "
                         "this invocation, outside the headline's timed region: deployment_* keys")
    ap.add_argument("--deployment-steps", type=int, default=3)
    ap.add_argument("--deployment-baseline-steps", type=int, default=2)
    ap.add_argument("--baseline-steps", type=int, default=2)
    ap.add_argument("--baseline-warmup", type=int, default=1)
    ap.add_argument("--payload-probe", choices=["auto", "cpu", "none"], default="auto",
                    help="after everything else, when the node has a GPU per rank, run the scheduled DDP "
                         "payload over RCCL on them (child process, time-limited) and report payload_ddp; "
                         "'cpu' runs it over gloo on the CPU (a rehearsal of the multi-rank path)")
    ap.add_argument("--payload-timeout", type=float, default=240.0)
    ap.add_argument("--lifecycle", choices=["realistic", "instant"], default="instant",
                    help="how each tick's jobs run before the next tick in the headline, single-process and "
                         "reference runs: 'instant' (default; the rounds 1-4 step, kept comparable) -- one "
                         "Succeeded write per job; 'realistic' -- the training-operator's status writes (Created, "
                         "one replicaStatuses write per pod, Running, Succeeded), each absorbed by the operator")
    ap.add_argument("--deployment-lifecycle", choices=["realistic", "instant"], default="realistic",
                    help="the same for the deployment-shaped pair (default realistic)")
    ap.add_argument("--completion-writes", choices=["interleaved", "batch"], default="interleaved",
                    help="instant lifecycle on the native fixture: the harness's job-completion writes are "
                         "applied a few per server loop turn between the operator's requests ('interleaved', as "
                         "at a real apiserver), or all in one call that holds the server for its length ('batch', "
                         "rounds 1-5); the fixture's CPU for them is inside the timed region either way")
    ap.add_argument("--out", default="", help="also write the full result JSON here")
    a = ap.parse_args()

    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_ranks(a.gpus)
    dist, rank, world = _dist()
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; refusing to report n_gpus={a.gpus}",
              file=sys.stderr)
        return 2
    from cron_operator_amd.bench.harness import LATENCY_PROFILES, BenchConfig, run_sync

    if a.shards <= 0:
        from cron_operator_amd.runtime.supervisor import available_cpus

        # never oversubscribe the CPUs the ranks share: with a partitioned fixture a core per shard
        # and per partition plus one (3 shards from 7 CPUs per rank, 2 from 5); otherwise a core
        # per shard plus one for the shared fake apiserver (3 shards saturate it)
        cpus = available_cpus() // world
        if a.fixture == "partitioned" and a.shard_routing == "labels" and a.transport == "http" and cpus >= 5:
            a.shards = min(3, (cpus - 1) // 2)
        else:
            a.shards = max(1, min(3, cpus - 1))

    from cron_operator_amd.runtime.supervisor import available_cpus

    shards = a.shards if a.transport == "http" else 1
    # a partitioned fixture: a fake apiserver process per shard, each with a core of its own
    can_partition = (shards > 1 and a.shard_routing == "labels"
                     and available_cpus() // world >= 2 * shards + 1)
    parts = shards if a.fixture == "partitioned" and can_partition else 1

    def bench_cfg(namespace: str, partitions: int) -> "BenchConfig":
        return BenchConfig(n_crons=a.crons, steps=a.steps, warmup=a.warmup, history_limit=a.history_limit,
                           mode=a.mode, transport=a.transport, qps=a.qps, burst=a.burst, workers=a.workers,
                           namespace=namespace, shards=shards, apiserver_partitions=partitions,
                           shard_routing=a.shard_routing, apiserver_latency=a.apiserver_latency, tls=a.tls,
                           max_inflight=a.max_inflight, defer_writes=not a.no_defer, lifecycle=a.lifecycle,
                           apiserver_impl=a.apiserver_impl, completion_writes=a.completion_writes)

    cfg = bench_cfg(f"bench-r{rank}", parts)

    def on_step(k: int, dt: float, timed: bool) -> None:
        # bracket the K timed steps with barriers so every rank times the same window: the
        # harness starts its clock right after step `warmup` returns and stops it after the
        # last step, i.e. after the closing barrier (which therefore counts: max over ranks)
        if k == cfg.warmup or k == cfg.warmup + cfg.steps:
            _sync_device()
            _barrier(dist)

    _barrier(dist)
    t0 = time.perf_counter()
    res = run_sync(cfg, on_step if cfg.warmup > 0 else None)
    _sync_device()
    _barrier(dist)
    wall = time.perf_counter() - t0
    _progress(rank, f"headline done: {cfg.n_crons * cfg.steps / res.elapsed_s:.1f} cron-reconciles/s "
                    f"(rank 0), {wall:.1f} s")

    mine = {"elapsed_s": res.elapsed_s, "fires": cfg.n_crons * cfg.steps,
            "reconciles": res.raw_reconciles_per_s * res.elapsed_s, "p50": res.p50_latency_ms,
            "p99": res.p99_latency_ms, "req_per_fire": res.api_requests_per_fire,
            "cpu_op": res.cpu_s_operator, "cpu_api_total": res.cpu_s_apiserver,
            # busy fraction: the busiest fake apiserver (one, or one per shard)
            "cpu_api": max(res.cpu_s_apiserver_parts) if res.cpu_s_apiserver_parts else res.cpu_s_apiserver,
            "shard_rss": max(res.operator_maxrss_mib or [0.0]), "shard_end_rss": max(res.operator_rss_mib or [0.0])}

    # the same shards against the other fixture layout (untimed for the headline)
    if a.other_fixture == "measure" and can_partition:
        ocfg = bench_cfg(f"bench-alt-r{rank}", 1 if parts > 1 else shards)
        _barrier(dist)
        try:
            ores = run_sync(ocfg)
        except Exception as e:  # noqa: BLE001 - an extra comparison must not cost the headline line
            ores = None
            mine["alt_error"] = f"{type(e).__name__}: {e}"[:300]
        _barrier(dist)
        if ores is not None:
            _progress(rank, f"{'shared' if parts > 1 else 'partitioned'} fixture done: "
                            f"{ocfg.n_crons * ocfg.steps / ores.elapsed_s:.1f}")
            mine["alt_elapsed_s"] = ores.elapsed_s
            mine["alt_fires"] = ocfg.n_crons * ocfg.steps
            mine["alt_p50"] = ores.p50_latency_ms
            mine["alt_cpu_op"] = ores.cpu_s_operator
            mine["alt_cpu_api"] = (max(ores.cpu_s_apiserver_parts) if ores.cpu_s_apiserver_parts
                                   else ores.cpu_s_apiserver)
        else:
            _progress(rank, f"other fixture failed: {mine['alt_error']}")

    # the shipped default: one operator process (untimed for the headline, like the baseline)
    if a.single_process == "measure" and a.transport == "http":
        if cfg.shards == 1:
            sres, scfg = res, cfg
        else:
            scfg = BenchConfig(n_crons=a.crons, steps=a.single_steps, warmup=a.single_warmup,
                               history_limit=a.history_limit, mode=a.mode, transport=a.transport, qps=a.qps,
                               burst=a.burst, workers=a.workers, namespace=f"bench-1p-r{rank}", shards=1,
                               apiserver_latency=a.apiserver_latency, tls=a.tls, max_inflight=a.max_inflight,
                               defer_writes=not a.no_defer, lifecycle=a.lifecycle, apiserver_impl=a.apiserver_impl,
                               completion_writes=a.completion_writes)
            _barrier(dist)
            sres = run_sync(scfg)
            _barrier(dist)
            _progress(rank, f"single process done: {scfg.n_crons * scfg.steps / sres.elapsed_s:.1f}")
        mine["sp_elapsed_s"] = sres.elapsed_s
        mine["sp_fires"] = scfg.n_crons * scfg.steps
        mine["sp_p50"] = sres.p50_latency_ms
        mine["sp_p99"] = sres.p99_latency_ms
        mine["sp_cpu_op"] = sres.cpu_s_operator
        mine["sp_cpu_api"] = sres.cpu_s_apiserver

    # the denominator: the reference algorithm on the same Crons, same box, same invocation
    # (untimed for the headline; one operator process, as the reference is one controller)
    if a.baseline == "measure":
        bcfg = BenchConfig(n_crons=a.crons, steps=a.baseline_steps, warmup=a.baseline_warmup,
                           history_limit=a.history_limit, mode="reference", transport=a.transport, qps=a.qps,
                           burst=a.burst, workers=a.workers, namespace=f"bench-ref-r{rank}", shards=1,
                           tls=a.tls, lifecycle=a.lifecycle, apiserver_impl=a.apiserver_impl,
                           completion_writes=a.completion_writes)
        _barrier(dist)
        bres = run_sync(bcfg)
        _barrier(dist)
        _progress(rank, f"reference algorithm done: {bcfg.n_crons * bcfg.steps / bres.elapsed_s:.1f}")
        mine["ref_elapsed_s"] = bres.elapsed_s
        mine["ref_fires"] = bcfg.n_crons * bcfg.steps
        mine["ref_p50"] = bres.p50_latency_ms
        mine["ref_req_per_fire"] = bres.api_requests_per_fire

    # deployment-shaped pair: TLS + etcd latency, one process, both algorithms (untimed for the headline)
    if a.deployment == "measure" and a.transport == "http":
        for tag, mode, steps in (("dep", "optimized", a.deployment_steps),
                                 ("dep_ref", "reference", a.deployment_baseline_steps)):
            dcfg = BenchConfig(n_crons=a.crons, steps=steps, warmup=1, history_limit=a.history_limit, mode=mode,
                               transport="http", qps=a.qps, burst=a.burst, workers=a.workers,
                               max_inflight=a.max_inflight, defer_writes=not a.no_defer,
                               namespace=f"bench-{tag.replace('_', '-')}-r{rank}", shards=1,
                               apiserver_latency="etcd", tls=True, lifecycle=a.deployment_lifecycle,
                               apiserver_impl=a.apiserver_impl, completion_writes=a.completion_writes)
            _barrier(dist)
            try:
                dres = run_sync(dcfg)
            except Exception as e:  # noqa: BLE001 - an extra comparison must not cost the headline line
                dres = None
                mine[f"{tag}_error"] = f"{type(e).__name__}: {e}"[:300]
            _barrier(dist)
            if dres is None:
                _progress(rank, f"deployment-shaped {mode} failed: {mine[f'{tag}_error']}")
                continue
            _progress(rank, f"deployment-shaped {mode} done: {dcfg.n_crons * dcfg.steps / dres.elapsed_s:.1f}")
            mine[f"{tag}_elapsed_s"] = dres.elapsed_s
            mine[f"{tag}_fires"] = dcfg.n_crons * dcfg.steps
            mine[f"{tag}_p50"] = dres.p50_latency_ms
            mine[f"{tag}_p99"] = dres.p99_latency_ms
            mine[f"{tag}_req_per_fire"] = dres.api_requests_per_fire
            mine[f"{tag}_cpu_api"] = dres.cpu_s_apiserver
            mine[f"{tag}_by_verb"] = dres.api_requests_by_verb
            mine[f"{tag}_reconciles_per_fire"] = dres.reconciles_per_fire
    # the scheduled payload over RCCL on this node's GPUs (untimed, last): rank 0 runs it while
    # the other ranks wait at the barrier, so no rank tears its process group down early
    probe = None
    if a.payload_probe != "none" and rank == 0:
        cpu = a.payload_probe == "cpu"
        _progress(rank, f"payload probe: DDP over {'gloo on the CPU' if cpu else f'RCCL on {world} GPU(s)'}, "
                        f"limit {a.payload_timeout:.0f} s")
        probe = (_payload_probe(world, a.payload_timeout, cpu=True, allreduce_mb=4, steps=2) if cpu
                 else _payload_probe(world, a.payload_timeout))
        _progress(rank, f"payload probe: {probe}")
    _barrier(dist)
    if dist is not None:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if rank == 0:
        t_max = max(r["elapsed_s"] for r in allr)  # timed region: max over ranks
        fires = sum(r["fires"] for r in allr)
        value = fires / t_max
        if a.baseline == "measure":
            base_value = sum(r["ref_fires"] for r in allr) / max(r["ref_elapsed_s"] for r in allr)
            base_src = (f"measured: reference algorithm (--mode reference, 1 process/rank), {a.baseline_steps} "
                        f"timed ticks, this invocation")
        elif a.baseline == "recorded":
            base_value, base_src = RECORDED_BASELINE_VALUE * world, "recorded: BASELINE.md r1i x ranks"
        else:
            base_value, base_src = None, "none"
        out = {
            "metric": "reconciles/sec + p50 schedule→create latency @1000 Cron CRs",
            "value": round(value, 2),
            "unit": "cron_reconciles/s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(t_max * 1000 / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base_value, 3) if base_value else None,
            "dtype": "n/a (control plane; no tensor compute)",
            "data": f"synthetic: {cfg.n_crons} random-free Cron CRs per rank (* * * * *, "
                    f"historyLimit={cfg.history_limit}) + PyTorchJob children on "
                    + (f"a fake apiserver process per shard ({cfg.apiserver_partitions} per rank, each holding its "
                       f"shard's Crons)" if cfg.apiserver_partitions > 1 else "a fake apiserver process per rank"),
            "config": {"model": "cron-operator Cron reconciler (apps.kubedl.io/v1alpha1)",
                       "global_batch": fires // a.steps, "seq_len": None,
                       "parallelism": f"ranks{world}x{cfg.shards}shards", "crons_per_rank": cfg.n_crons,
                       "history_limit": cfg.history_limit, "schedule": "* * * * *",
                       "transport": cfg.transport, "mode": cfg.mode, "workers": cfg.workers,
                       "operator_shards": cfg.shards,
                       "shard_routing": cfg.shard_routing if cfg.shards > 1 else None,
                       "apiserver_latency": cfg.apiserver_latency,
                       "tls": cfg.tls, "qps": cfg.qps, "job_lifecycle": cfg.lifecycle,
                       "apiserver_impl": cfg.apiserver_impl, "completion_writes": cfg.completion_writes,
                       "fixture": "partitioned" if cfg.apiserver_partitions > 1 else "shared",
                       "apiserver_partitions": cfg.apiserver_partitions,
                       # CPUs the job may use per rank (cgroup quota / affinity): what chose shards and fixture
                       "cpus_per_rank": available_cpus() // world},
            "p50_schedule_to_create_ms": round(max(r["p50"] for r in allr), 2),
            "p99_schedule_to_create_ms": round(max(r["p99"] for r in allr), 2),
            "raw_reconciles_per_s": round(sum(r["reconciles"] for r in allr) / t_max, 2),
            "api_requests_per_fire": round(sum(r["req_per_fire"] for r in allr) / len(allr), 3),
            # operator-side cost (all shard processes), the number to track rather than the
            # fake apiserver's speed; and how busy that fixture was (CPU s / wall s, max rank)
            "operator_cpu_ms_per_fire": round(sum(r["cpu_op"] for r in allr) * 1000 / fires, 4),
            # (the busiest fake apiserver of any rank: with a partitioned fixture, its busiest partition)
            "apiserver_busy_frac": round(max(r["cpu_api"] / r["elapsed_s"] for r in allr), 3),
            # the fixture's own CPU per fire (all ranks' fake apiservers): its speed, apart from the load
            "apiserver_cpu_us_per_fire": round(sum(r["cpu_api_total"] for r in allr) * 1e6 / fires, 1),
            # peak resident memory (VmHWM) of the largest operator shard process (0: the operator
            # ran in the bench process itself)
            "operator_shard_peak_rss_mib": round(max(r.get("shard_rss", 0.0) for r in allr), 1),
            # ... and the largest shard's resident size at the end of the run (peak >= end)
            "operator_shard_end_rss_mib": round(max(r.get("shard_end_rss", 0.0) for r in allr), 1),
            "baseline_value": round(base_value, 2) if base_value else None,
            "baseline_source": base_src,
            "baseline_p50_schedule_to_create_ms": round(max(r["ref_p50"] for r in allr), 2)
            if a.baseline == "measure" else None,
            # the fixture-independent comparison: API requests per fire of each algorithm (under a
            # client QPS limit, throughput is QPS / requests per fire)
            "baseline_api_requests_per_fire": round(sum(r["ref_req_per_fire"] for r in allr) / len(allr), 3)
            if a.baseline == "measure" else None,
            "cron_engine": res.engine,
            "wall_s": round(wall, 2),
        }
        # the headline's shards against the other fixture layout: shared_fixture_* when the
        # headline is partitioned (rounds 1-5's layout, one fake apiserver for every shard), else
        # partitioned_*
        alt = "shared_fixture" if cfg.apiserver_partitions > 1 else "partitioned"
        alt_errors = sorted({r["alt_error"] for r in allr if "alt_error" in r})
        if alt_errors:
            out[f"{alt}_error"] = "; ".join(alt_errors)
        elif all("alt_fires" in r for r in allr):
            alt_fires = sum(r["alt_fires"] for r in allr)
            out.update({
                f"{alt}_value": round(alt_fires / max(r["alt_elapsed_s"] for r in allr), 2),
                f"{alt}_p50_ms": round(max(r["alt_p50"] for r in allr), 2),
                f"{alt}_operator_cpu_ms_per_fire": round(sum(r["alt_cpu_op"] for r in allr) * 1000 / alt_fires, 4),
                # the busiest fake apiserver of any rank (CPU s / wall s)
                f"{alt}_apiserver_busy_frac": round(max(r["alt_cpu_api"] / r["alt_elapsed_s"] for r in allr), 3),
            })
        if "sp_fires" in allr[0]:
            sp_fires = sum(r["sp_fires"] for r in allr)
            out.update({
                # the chart's default deployment: one operator process per rank, same Crons
                "single_process_value": round(sp_fires / max(r["sp_elapsed_s"] for r in allr), 2),
                "single_process_p50_ms": round(max(r["sp_p50"] for r in allr), 2),
                "single_process_p99_ms": round(max(r["sp_p99"] for r in allr), 2),
                "single_process_operator_cpu_ms_per_fire": round(sum(r["sp_cpu_op"] for r in allr) * 1000
                                                                 / sp_fires, 4),
                "single_process_apiserver_busy_frac": round(max(r["sp_cpu_api"] / r["sp_elapsed_s"]
                                                                for r in allr), 3),
            })
        dep_errors = sorted({r[k] for r in allr for k in ("dep_error", "dep_ref_error") if k in r})
        if dep_errors:
            out["deployment_error"] = "; ".join(dep_errors)
        elif all("dep_fires" in r and "dep_ref_fires" in r for r in allr) and allr[0].get("dep_fires"):
            dv = sum(r["dep_fires"] for r in allr) / max(r["dep_elapsed_s"] for r in allr)
            dbv = sum(r["dep_ref_fires"] for r in allr) / max(r["dep_ref_elapsed_s"] for r in allr)
            out.update({
                "deployment_config": {"operator_processes": 1, "tls": True, "apiserver_latency": "etcd",
                                      "latency_model_s": LATENCY_PROFILES["etcd"],
                                      "workers": a.workers, "qps": a.qps,
                                      "job_lifecycle": a.deployment_lifecycle},
                "deployment_value": round(dv, 2),
                "deployment_p50_ms": round(max(r["dep_p50"] for r in allr), 2),
                "deployment_p99_ms": round(max(r["dep_p99"] for r in allr), 2),
                "deployment_api_requests_per_fire": round(sum(r["dep_req_per_fire"] for r in allr) / len(allr), 3),
                "deployment_baseline_value": round(dbv, 2),
                "deployment_baseline_p50_ms": round(max(r["dep_ref_p50"] for r in allr), 2),
                "deployment_baseline_api_requests_per_fire": round(
                    sum(r["dep_ref_req_per_fire"] for r in allr) / len(allr), 3),
                "vs_baseline_deployment": round(dv / dbv, 3) if dbv else None,
                # both arms must be latency-bound, not fixture-bound: the fake apiserver's CPU
                # seconds per wall second over each arm's timed region (max over ranks)
                "deployment_apiserver_busy_frac": round(max(r["dep_cpu_api"] / r["dep_elapsed_s"] for r in allr), 3),
                "deployment_baseline_apiserver_busy_frac": round(
                    max(r["dep_ref_cpu_api"] / r["dep_ref_elapsed_s"] for r in allr), 3),
                "deployment_reconciles_per_fire": round(sum(r["dep_reconciles_per_fire"] for r in allr) / len(allr), 3),
                "deployment_baseline_reconciles_per_fire": round(
                    sum(r["dep_ref_reconciles_per_fire"] for r in allr) / len(allr), 3),
                # the reference algorithm's analytical ceiling under the same latency model: each
                # of its `workers` reconciles awaits its requests in turn, so it cannot exceed
                # workers / (model latency of its requests per fire) fires/s per rank
                "deployment_baseline_latency_ceiling": _latency_ceiling(allr, a.workers, a.crons,
                                                                         a.history_limit, LATENCY_PROFILES["etcd"]),
            })
        if probe is not None:
            out["payload_ddp"] = probe
        print(json.dumps(out), flush=True)
        if a.out:
            with open(a.out, "w") as fh:
                json.dump({"summary": out, "rank0": res.to_dict()}, fh, indent=1)
    if dist is not None:
        # every rank is past its last collective (and rank 0 has printed) before any rank tears
        # its gloo connections down: a peer closing early can abort a rank still reading
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
