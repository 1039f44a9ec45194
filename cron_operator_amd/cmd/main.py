"""Command line: ``cron-operator start [flags]`` and helper subcommands.

Reference: ``cmd/main.go:31-55`` (cobra root that prints help without a
subcommand) and ``cmd/operator/start.go:61-265`` (the ``start`` command).  Every
flag of the reference keeps its name and meaning, and every default but two: ``--qps`` /
``--burst`` ship 150 / 300 instead of 30 / 50 (sized for 1000+ minutely Crons; a drop-in
switch-over may send up to 5x the reference's client-side request rate, see
docs/migration.md "Changed defaults").  ``--max-concurrent-reconciles`` bounds the reconciles
*deciding* at once; a reconcile left with only API writes hands its slot on, and up to
``max(1024, 100 x N)`` of those may be writing (``runtime/controller.py``):

==============================  ===========  ==========================================
flag                            default      reference
==============================  ===========  ==========================================
--max-concurrent-reconciles     10           start.go:215
--qps / --burst                 150 / 300    start.go:218-219 (30 / 50 there; sized here for 1000+
                                             minutely Crons, see docs/operations.md "Sizing qps")
--metrics-bind-address          "0"          start.go:220 (0 disables)
--health-probe-bind-address     ":8081"      start.go:222
--leader-elect                  false        start.go:223
--metrics-secure                true         start.go:226
--webhook-cert-path/-name/-key  ""/tls.crt/tls.key   start.go:228-234
--metrics-cert-path/-name/-key  ""/tls.crt/tls.key   start.go:235-240
--enable-http2                  false        start.go:241
--zap-devel/-encoder/-log-level/-stacktrace-level/-time-encoding      start.go:244-247
==============================  ===========  ==========================================

Additions: ``--kubeconfig``, ``--namespace`` (restrict the cache),
``--leader-elect-namespace``, ``--compat-mode`` (``reference`` restores every
reference quirk, see :class:`~cron_operator_amd.controller.reconciler.ReconcilerOptions`),
``--cron-engine``, ``--max-inflight-requests``, ``--tick-burst-reserve``.  Extra subcommands:
``fake-apiserver`` (serve the in-process apiserver over HTTP with the CRDs installed), ``crd``
(print the CRD) and ``version``.

Flag syntax follows pflag: ``--flag value``, ``--flag=value`` and bare boolean
flags (``--leader-elect``, ``--metrics-secure=false``).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import sys
from typing import Any, List, Optional

from .. import __version__


def _bool(v: Optional[str]) -> bool:
    if v is None:
        return True
    s = str(v).strip().lower()
    if s in ("1", "t", "true", "yes", "y", "on"):
        return True
    if s in ("0", "f", "false", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError(f'invalid boolean value "{v}"')


def _add_bool(p: argparse.ArgumentParser, name: str, default: bool, help_: str) -> None:
    p.add_argument(name, nargs="?", const=True, default=default, type=_bool, metavar="true|false", help=help_)


def _processes(v: str) -> int:
    if v == "auto":
        from ..runtime.supervisor import available_cpus

        return available_cpus()
    try:
        return int(v)
    except ValueError:
        raise argparse.ArgumentTypeError(f"invalid --shard-processes {v!r} (an integer or 'auto')") from None


# client sizing (docs/operations.md "Sizing qps"): ~4 requests per Cron fire.  Measured at 150 /
# 300 (profiles/chart_defaults_mi355x_box_r5.json): 1000 minutely Crons take 28.7 s of each 60 s
# tick, p50 tick->create 1.35 s; 2000 take 57.4 s, p50 4.7 s -- one slow tick from collapse, so
# `preflight` warns past 80% of the minute (~1800 Crons).  The burst absorbs a tick's first
# CREATEs.  The reference ships 30 / 50 (start.go:218-219), which tops out near 450 Crons.
DEFAULT_QPS = 150.0
DEFAULT_BURST = 300
DEFAULT_MAX_INFLIGHT = 128


def build_parser() -> argparse.ArgumentParser:
    root = argparse.ArgumentParser(prog="cron-operator", description="Cron operator for scheduled ML training jobs "
                                                                     "(apps.kubedl.io/v1alpha1 Cron).")
    sub = root.add_subparsers(dest="command")

    st = sub.add_parser("start", help="Start manager")
    st.add_argument("--max-concurrent-reconciles", type=int, default=10,
                    help="The maximum number of concurrent reconciles for controller (reconciles deciding "
                         "at once; one left with only API writes hands its slot on, and up to max(1024, 100 x "
                         "this) such reconciles may be writing, their requests bounded by --qps and "
                         "--max-inflight-requests).")
    st.add_argument("--qps", type=float, default=DEFAULT_QPS,
                    help="Maximum QPS to the Kubernetes API server from this client. About 4 requests per Cron "
                         "fire: N minutely Crons need N/15 QPS (default: 1000 Crons at 45%% of the budget).")
    st.add_argument("--burst", type=int, default=DEFAULT_BURST, help="Maximum burst for throttle.")
    st.add_argument("--tick-burst-reserve", type=int, default=-1,
                    help="Burst tokens that deferrable writes (status PATCHes, history-GC DELETEs, events) may "
                         "not spend: they run at the --qps refill rate and leave the burst to the next schedule "
                         "tick's CREATEs. -1 (default): the whole burst; 0: off.")
    st.add_argument("--max-inflight-requests", type=int, default=DEFAULT_MAX_INFLIGHT,
                    help="Maximum concurrent API requests (watches excluded); more wait in priority order "
                         "(tick CREATEs first). 0: unlimited.")
    st.add_argument("--metrics-bind-address", default="0", help="The address the metrics endpoint binds to. Use "
                                                                ":8443 for HTTPS or :8080 for HTTP, or leave as 0 to "
                                                                "disable the metrics service.")
    st.add_argument("--health-probe-bind-address", default=":8081", help="The address the probe endpoint binds to.")
    _add_bool(st, "--leader-elect", False, "Enable leader election for controller manager. Enabling this will "
                                           "ensure there is only one active controller manager.")
    _add_bool(st, "--metrics-secure", True, "If set, the metrics endpoint is served securely via HTTPS. Use "
                                            "--metrics-secure=false to use HTTP instead.")
    st.add_argument("--webhook-cert-path", default="", help="The directory that contains the webhook certificate.")
    st.add_argument("--webhook-cert-name", default="tls.crt", help="The name of the webhook certificate file.")
    st.add_argument("--webhook-cert-key", default="tls.key", help="The name of the webhook key file.")
    st.add_argument("--metrics-cert-path", default="", help="The directory that contains the metrics server "
                                                            "certificate.")
    st.add_argument("--metrics-cert-name", default="tls.crt", help="The name of the metrics server certificate file.")
    st.add_argument("--metrics-cert-key", default="tls.key", help="The name of the metrics server key file.")
    _add_bool(st, "--enable-http2", False, "If set, HTTP/2 will be enabled for the metrics and webhook servers")
    # zap flags (controller-runtime logzap.Options.BindFlags)
    _add_bool(st, "--zap-devel", False, "Development Mode defaults(encoder=consoleEncoder,logLevel=Debug,"
                                        "stackTraceLevel=Warn). Production Mode defaults(encoder=jsonEncoder,"
                                        "logLevel=Info,stackTraceLevel=Error)")
    st.add_argument("--zap-encoder", default=None, help="Zap log encoding (one of 'json' or 'console')")
    st.add_argument("--zap-log-level", default=None, help="Zap Level to configure the verbosity of logging. Can be "
                                                          "one of 'debug', 'info', 'error', 'panic'or any integer "
                                                          "value > 0 which corresponds to custom debug levels of "
                                                          "increasing verbosity")
    st.add_argument("--zap-stacktrace-level", default=None, help="Zap Level at and above which stacktraces are "
                                                                 "captured (one of 'info', 'error', 'panic').")
    st.add_argument("--zap-time-encoding", default=None, help="Zap time encoding (one of 'epoch', 'millis', 'nano', "
                                                              "'iso8601', 'rfc3339' or 'rfc3339nano'). Defaults to "
                                                              "'epoch'.")
    # additions
    st.add_argument("--kubeconfig", default="", help="Path to a kubeconfig. Only required if out-of-cluster.")
    st.add_argument("--namespace", default="", help="Only watch Crons in this namespace (default: all).")
    st.add_argument("--leader-elect-namespace", default="", help="Namespace of the leader-election Lease "
                                                                 "(default: the pod's namespace).")
    st.add_argument("--compat-mode", choices=["optimized", "reference"], default="optimized",
                    help="'reference' reproduces every reference behaviour (live child LIST, finished=now, ...).")
    st.add_argument("--cron-engine", choices=["auto", "native", "python"], default="auto",
                    help="Cron next-fire engine implementation.")
    st.add_argument("--shard-count", type=int, default=1, help="Split Crons across this many operator "
                                                                "replicas (hash of namespace/name).")
    st.add_argument("--shard-index", type=int, default=int(os.environ.get("SHARD_INDEX", "0") or 0),
                    help="This replica's shard in [0, --shard-count) (default: $SHARD_INDEX).")
    st.add_argument("--shard-processes", type=_processes, default=1,
                    help="Run this many operator processes in this pod, one shard each (the pod's share of "
                         "--shard-count is split further), under a supervisor that serves the merged metrics "
                         "and the probes. Uses that many cores, like the reference's goroutine workers. "
                         "'auto': the CPUs the container may use (cgroup quota, else affinity).")
    st.add_argument("--shard-routing", choices=["hash", "labels"], default="labels",
                    help="Only when sharded. labels (default): shards label their Crons and children "
                         "kubedl.io/shard=<index>-of-<count> and watch only their own (the apiserver splits "
                         "the watch traffic; the configuration the benchmarks measure); hash: every shard "
                         "watches all objects and drops other shards' keys (no labels written).")
    st.add_argument("--sync-period", default="10h", help="Minimum frequency at which every watched object is "
                                                        "reconciled again (controller-runtime's cache SyncPeriod; "
                                                        "Go duration, 0 disables).")
    _add_bool(st, "--enable-tracing", False, "Record per-reconcile spans (served at /debug/traces on the probe port).")
    st.add_argument("--trace-file", default="", help="Also append finished spans here as JSON lines "
                                                     "(implies --enable-tracing).")
    st.add_argument("--trace-sample-rate", type=float, default=1.0, help="Fraction of reconciles traced.")
    _add_bool(st, "--enable-profiling", False, "Serve a CPU profile of the event loop at "
                                              "/debug/profile?seconds=N on the probe port.")
    st.add_argument("--debug-views", choices=["local", "all", "off"], default="local",
                    help="Who may read the probe port's /debug views (/debug/caches, /debug/tasks, "
                         "/debug/traces, /debug/profile): local (default) -- loopback clients only, e.g. "
                         "kubectl port-forward; all -- any client (cover the port with a NetworkPolicy); off.")

    fa = sub.add_parser("fake-apiserver", help="Serve the in-process fake Kubernetes API server over HTTP")
    fa.add_argument("--bind-address", default="127.0.0.1")
    fa.add_argument("--port", type=int, default=6443)
    fa.add_argument("--kubeconfig-out", default="", help="Write a kubeconfig pointing at the server here.")
    _add_bool(fa, "--gc", True, "Run ownerReference garbage collection.")
    _add_bool(fa, "--fake-clock", False, "Use a settable clock (POST /debug/fake/clock).")
    fa.add_argument("--token", default="", help="Require this bearer token (an admin: group system:masters).")
    fa.add_argument("--sa-token", action="append", default=[], metavar="TOKEN=NAMESPACE:NAME",
                    help="Also accept TOKEN as ServiceAccount NAMESPACE/NAME (repeatable).")
    fa.add_argument("--authorization-mode", choices=["AlwaysAllow", "RBAC"], default="AlwaysAllow",
                    help="RBAC: authorize requests against stored (Cluster)Roles and bindings.")
    _add_bool(fa, "--training-operator", False, "Also run the fake training-operator (timed mode).")
    fa.add_argument("--job-duration", type=float, default=30.0, help="Seconds a job runs in timed mode.")

    gt = sub.add_parser("get", help="List Crons (or one Cron) like `kubectl get crons`")
    gt.add_argument("resource", nargs="?", default="crons", help="crons | cron (kubectl aliases accepted)")
    gt.add_argument("name", nargs="?", default="")
    gt.add_argument("-n", "--namespace", default="default")
    gt.add_argument("-A", "--all-namespaces", action="store_true")
    gt.add_argument("-l", "--selector", default="")
    gt.add_argument("-o", "--output", default="", choices=["", "wide", "json", "yaml", "name"])
    gt.add_argument("--kubeconfig", default="")
    gt.add_argument("--no-headers", action="store_true")
    sub.add_parser("crd", help="Print the Cron CustomResourceDefinition")
    kz = sub.add_parser("kustomize", help="Render a kustomization directory (kustomize build)")
    kz.add_argument("dir", nargs="?", default="deploy/kustomize/default")
    kz.add_argument("-o", "--output", default="", help="Write here instead of stdout (e.g. dist/install.yaml).")
    kz.add_argument("--enable-optional", action="store_true",
                    help="Render with every commented-out optional section enabled (cert-manager metrics "
                         "certificate, ServiceMonitor with TLS verification, network policy)")
    hm = sub.add_parser("helm-template", help="Render the Helm chart (helm template)")
    hm.add_argument("chart", nargs="?", default="charts/cron-operator")
    hm.add_argument("--release", default="cron-operator")
    hm.add_argument("--namespace", default="cron-operator")
    hm.add_argument("--set", action="append", default=[], help="key.path=value overrides")
    hm.add_argument("-f", "--values", action="append", default=[], help="values file(s)")
    sub.add_parser("version", help="Print the version")
    from .preflight import add_parser as add_preflight

    add_preflight(sub)
    return root


def _setup_log(a: argparse.Namespace):
    from ..utils.logging import new_from_options, set_logger

    logger = new_from_options(encoder=a.zap_encoder, level=a.zap_log_level, devel=a.zap_devel,
                              stacktrace_level=a.zap_stacktrace_level, time_encoding=a.zap_time_encoding)
    set_logger(logger)
    return logger


async def run_start(a: argparse.Namespace) -> int:
    from ..controller.reconciler import ReconcilerOptions
    from ..controller.setup import setup_with_manager
    from ..cron.engine import make_engine
    from ..runtime.client import Client
    from ..runtime.http import HttpTransport
    from ..runtime.kubeconfig import ConfigError, get_config
    from ..runtime.manager import LeaderElectionLost, Manager, ManagerOptions
    from ..utils.logging import get_logger

    log = get_logger("setup")
    if a.enable_profiling:
        from ..runtime import profiler

        profiler.allow()
    if a.enable_tracing or a.trace_file:
        from ..runtime import tracing

        tracing.set_tracer(tracing.Tracer(enabled=True, sample_rate=a.trace_sample_rate, file=a.trace_file))
        log.info("tracing enabled", sampleRate=a.trace_sample_rate, file=a.trace_file or None)
    if not a.enable_http2:
        log.info("disabling http/2")
    if a.webhook_cert_path:
        log.info("Initializing webhook certificate watcher using provided certificates",
                 **{"webhook-cert-path": a.webhook_cert_path, "webhook-cert-name": a.webhook_cert_name,
                    "webhook-cert-key": a.webhook_cert_key})
    if a.metrics_cert_path:
        log.info("Initializing metrics certificate watcher using provided certificates",
                 **{"metrics-cert-path": a.metrics_cert_path, "metrics-cert-name": a.metrics_cert_name,
                    "metrics-cert-key": a.metrics_cert_key})
    try:
        cfg = get_config(a.kubeconfig)
    except ConfigError as e:
        log.error(e, "unable to get kubeconfig")
        return 1
    if a.shard_count < 1 or not 0 <= a.shard_index < a.shard_count:
        log.error(ValueError(f"--shard-index {a.shard_index} not in [0, {a.shard_count})"), "invalid sharding")
        return 2
    cfg.qps, cfg.burst = a.qps, a.burst
    from ..utils.gotime import NANOS, parse_duration

    try:
        sync_period = parse_duration(a.sync_period) / NANOS if a.sync_period not in ("", "0") else 0.0
    except ValueError as e:
        log.error(e, "invalid --sync-period")
        return 2
    client = Client(HttpTransport(cfg, pool_size=max(64, a.max_inflight_requests)), qps=a.qps, burst=a.burst,
                    max_inflight=a.max_inflight_requests, low_reserve=a.tick_burst_reserve)
    mopts = ManagerOptions(namespace=a.namespace, leader_election=a.leader_elect,
                           leader_election_namespace=a.leader_elect_namespace,
                           metrics_bind_address=a.metrics_bind_address, secure_metrics=a.metrics_secure,
                           metrics_cert_path=a.metrics_cert_path, metrics_cert_name=a.metrics_cert_name,
                           metrics_cert_key=a.metrics_cert_key,
                           health_probe_bind_address=a.health_probe_bind_address, debug_views=a.debug_views,
                           enable_http2=a.enable_http2, max_concurrent_reconciles=a.max_concurrent_reconciles,
                           sync_period=sync_period, shard_index=a.shard_index, shard_count=a.shard_count,
                           shard_routing=a.shard_routing)
    try:
        mgr = Manager(client, mopts)
        opts = ReconcilerOptions.reference() if a.compat_mode == "reference" else ReconcilerOptions()
        await setup_with_manager(mgr, opts, make_engine(a.cron_engine))
    except Exception as e:  # noqa: BLE001
        log.error(e, "unable to create controller", controller="Cron")
        await client.close()
        return 1
    mgr.add_healthz_check("healthz")
    mgr.add_readyz_check("readyz")
    loop = asyncio.get_running_loop()
    signals = [0]

    def on_signal() -> None:
        # ctrl.SetupSignalHandler: the first SIGTERM/SIGINT stops the manager gracefully,
        # a second one exits at once with status 1
        signals[0] += 1
        if signals[0] > 1:
            os._exit(1)
        mgr.stop()

    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, on_signal)
        except (NotImplementedError, RuntimeError):
            pass
    from ..ops import aioloop_native, netconn_native

    log.info("starting manager", **{"event loop": aioloop_native.status(),
                                    "http connections": netconn_native.status()})
    try:
        await mgr.start()
    except LeaderElectionLost:
        log.info("leader election lost")
        return 1
    except Exception as e:  # noqa: BLE001
        log.error(e, "problem running manager")
        return 1
    finally:
        await client.close()
    return 0


async def run_supervisor(a: argparse.Namespace, argv: List[str]) -> int:
    """``start --shard-processes N`` (runtime/supervisor.py)."""
    from ..runtime.client import Client
    from ..runtime.http import HttpTransport
    from ..runtime.kubeconfig import ConfigError, get_config
    from ..runtime.servers import MetricsServer, parse_bind_address
    from ..runtime.supervisor import Supervisor
    from ..utils.logging import get_logger

    log = get_logger("setup")
    if a.shard_count < 1 or not 0 <= a.shard_index < a.shard_count:
        log.error(ValueError(f"--shard-index {a.shard_index} not in [0, {a.shard_count})"), "invalid sharding")
        return 2
    client = None
    metrics = None
    if parse_bind_address(a.metrics_bind_address) is not None:
        if a.metrics_secure:  # TokenReview / SubjectAccessReview need the API
            try:
                cfg = get_config(a.kubeconfig)
            except ConfigError as e:
                log.error(e, "unable to get kubeconfig")
                return 1
            client = Client(HttpTransport(cfg, pool_size=max(64, a.max_inflight_requests)), qps=a.qps, burst=a.burst,
                            max_inflight=a.max_inflight_requests)
        metrics = MetricsServer(a.metrics_bind_address, secure=a.metrics_secure, cert_dir=a.metrics_cert_path,
                                cert_name=a.metrics_cert_name, key_name=a.metrics_cert_key, client=client,
                                enable_http2=a.enable_http2)
    sup = Supervisor(argv, a.shard_processes, a.shard_count, a.shard_index, metrics, a.health_probe_bind_address,
                     a.debug_views)
    log.info("starting shard processes", processes=a.shard_processes,
             shards=[c.index for c in sup.children], shardCount=a.shard_count * a.shard_processes)
    try:
        return await sup.run()
    finally:
        if client is not None:
            await client.close()


async def run_fake_apiserver(a: argparse.Namespace) -> int:
    from ..api.v1alpha1.crd import crd
    from ..apiserver.http import APIServerApp
    from ..apiserver.server import APIServer
    from ..runtime.client import Client, InMemoryTransport
    from ..runtime.kubeconfig import write_kubeconfig
    from ..trainingop.crds import kubeflow_crds
    from ..trainingop.operator import FakeTrainingOperator
    from ..utils.clock import FakeClock, RealClock

    clock = FakeClock() if a.fake_clock else RealClock()
    from ..apiserver.rbac import service_account_user

    tokens = {a.token: {"username": "admin", "groups": ["system:masters"]}} if a.token else None
    for spec in a.sa_token:
        tok, _, who = spec.partition("=")
        ns, _, name = who.partition(":")
        if not (tok and ns and name):
            print(f"invalid --sa-token {spec!r} (want TOKEN=NAMESPACE:NAME)", file=sys.stderr)
            return 2
        tokens = tokens or {}
        tokens[tok] = service_account_user(ns, name)
    server = APIServer(clock, gc=a.gc, tokens=tokens, authorization=a.authorization_mode)
    server.install_crd(crd())
    for c in kubeflow_crds():
        server.install_crd(c)
    app = APIServerApp(server)
    port = await app.start(a.bind_address, a.port)
    url = f"http://{a.bind_address}:{port}"
    if a.kubeconfig_out:
        write_kubeconfig(a.kubeconfig_out, url, a.token)
    print(f"fake apiserver listening on {url}", flush=True)
    top = None
    if a.training_operator:
        top = FakeTrainingOperator(Client(InMemoryTransport(server), qps=-1), clock, mode="timed",
                                   duration=a.job_duration)
        await top.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    await stop.wait()
    if top is not None:
        await top.stop()
    await app.stop()
    return 0


async def run_get(a: argparse.Namespace) -> int:
    import yaml

    from ..api import errors
    from ..api.v1alpha1 import CRON_GVR
    from ..apiserver.table import render
    from ..runtime.client import Client
    from ..runtime.http import HttpTransport
    from ..runtime.kubeconfig import ConfigError, get_config

    if a.resource.lower() not in ("crons", "cron", "crons.apps.kubedl.io", "cron.apps.kubedl.io"):
        print(f'error: the server doesn\'t have a resource type "{a.resource}"', file=sys.stderr)
        return 1
    try:
        cfg = get_config(a.kubeconfig)
    except ConfigError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    client = Client(HttpTransport(cfg), qps=-1)
    ns = "" if a.all_namespaces else a.namespace
    try:
        if a.output in ("json", "yaml", "name"):
            if a.name:
                data: Any = await client.get(CRON_GVR, ns, a.name)
                items = [data]
            else:
                data = await client.list(CRON_GVR, ns, a.selector or None)
                items = data.get("items") or []
            if a.output == "name":
                sys.stdout.write("".join(f"cron.apps.kubedl.io/{o['metadata']['name']}\n" for o in items))
            elif a.output == "json":
                sys.stdout.write(json.dumps(data, indent=4) + "\n")
            else:
                sys.stdout.write(yaml.safe_dump(data, sort_keys=False))
            return 0
        table = await client.table(CRON_GVR, ns, a.name, a.selector or None)
        if not table.get("rows"):
            where = "any namespace" if a.all_namespaces else f"{ns} namespace"
            print(f"No resources found in {where}.", file=sys.stderr)
            return 0
        sys.stdout.write(render(table, wide=a.output == "wide", namespace_column=a.all_namespaces,
                                no_headers=a.no_headers))
        return 0
    except errors.ApiError as e:
        print(f"Error from server ({e.reason}): {e.message}", file=sys.stderr)
        return 1
    finally:
        await client.close()


def _helm_template(a: argparse.Namespace) -> int:
    import yaml

    from ..utils.gotemplate import render_chart

    values: dict = {}

    def put(path: str, val) -> None:
        cur = values
        keys = path.split(".")
        for k in keys[:-1]:
            cur = cur.setdefault(k, {})
        cur[keys[-1]] = val

    def merge(dst: dict, src: dict) -> None:
        for k, v in src.items():
            if isinstance(v, dict) and isinstance(dst.get(k), dict):
                merge(dst[k], v)
            else:
                dst[k] = v

    for f in a.values:
        with open(f) as fh:
            merge(values, yaml.safe_load(fh) or {})
    for kv in a.set:
        k, _, v = kv.partition("=")
        put(k, yaml.safe_load(v) if v else "")
    docs = render_chart(a.chart, values, release=a.release, namespace=a.namespace)
    for name, objs in docs.items():
        for obj in objs:
            sys.stdout.write(f"---\n# Source: {name}\n" + yaml.safe_dump(obj, sort_keys=False))
    return 0


SUBCOMMANDS = ("start", "fake-apiserver", "get", "crd", "kustomize", "helm-template", "version", "preflight")


def cobra_order(argv: List[str]) -> List[str]:
    """Accept a subcommand's flags before its name, as cobra does: it strips leading flags to
    find the subcommand, which then parses every remaining flag.  The reference's kustomize
    tree relies on it -- its metrics patch inserts ``--metrics-bind-address=:8443`` at
    ``args[0]``, ahead of ``start`` (``config/default/manager_metrics_patch.yaml``)."""
    if not argv or not argv[0].startswith("-") or argv[0] in ("-h", "--help"):
        return list(argv)
    for i, tok in enumerate(argv):
        if tok in SUBCOMMANDS:
            return [tok] + list(argv[:i]) + list(argv[i + 1:])
    return list(argv)


def main(argv: Optional[List[str]] = None) -> int:
    parser = build_parser()
    argv = cobra_order(sys.argv[1:] if argv is None else argv)
    a = parser.parse_args(argv)
    if a.command is None:
        parser.print_help()
        return 0
    if a.command == "version":
        print(__version__)
        return 0
    if a.command == "crd":
        from ..api.v1alpha1.crd import crd_yaml

        sys.stdout.write(crd_yaml())
        return 0
    if a.command == "get":
        return asyncio.run(run_get(a))
    if a.command == "preflight":
        from .preflight import run as run_preflight

        return asyncio.run(run_preflight(a))
    if a.command == "kustomize":
        from ..utils.kustomize import build_yaml, enable_optional

        if a.enable_optional:
            import tempfile

            with tempfile.TemporaryDirectory() as tmp:
                out = build_yaml(enable_optional(a.dir, os.path.join(tmp, "tree")))
        else:
            out = build_yaml(a.dir)
        if a.output:
            os.makedirs(os.path.dirname(a.output) or ".", exist_ok=True)
            with open(a.output, "w") as fh:
                fh.write(out)
        else:
            sys.stdout.write(out)
        return 0
    if a.command == "helm-template":
        return _helm_template(a)
    if a.command == "fake-apiserver":
        return asyncio.run(run_fake_apiserver(a))
    if a.command == "start":
        try:
            _setup_log(a)
        except ValueError as e:
            print(f"invalid argument: {e}", file=sys.stderr)
            return 2
        if a.cron_engine != "auto":
            os.environ["CRON_OPERATOR_ENGINE"] = a.cron_engine
        from ..runtime import aioloop

        aioloop.install()  # the operator's loop: native call_soon/_run_once (runtime/aioloop.py)
        if a.shard_processes > 1:
            return asyncio.run(run_supervisor(a, list(argv)))
        if a.shard_processes < 1:
            print("invalid argument: --shard-processes must be >= 1", file=sys.stderr)
            return 2
        return asyncio.run(run_start(a))
    parser.print_help()
    return 2


if __name__ == "__main__":
    sys.exit(main())
