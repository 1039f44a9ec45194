"""``cron-operator preflight``: check a cluster before this operator takes it over.

A cluster run by the reference operator (or by this one, before an upgrade) holds Crons
whose templates name workload kinds.  Before switching (``docs/migration.md``), this reads
the cluster with the caller's kubeconfig -- nothing is written -- and reports, per kind the
templates use, whether the apiserver serves it and whether the operator's RBAC
(``controller/rbac.py`` ``RULES``, as the chart and kustomize installs grant it, plus any
``rbac.extraWorkloadRules``) lets it create, watch and delete that kind; every schedule
that does not parse (the reference's ``cron.ParseStandard`` grammar,
``internal/controller/cron_controller.go:184-190``); templates that set ``metadata.name``
(the reference's ``OverridePolicy``: such a Cron runs as Forbid, ``cron_controller.go:355-370``);
and who holds the leader Lease.  Exit status 1 when a Cron would fail to run.

It also sizes the client budget (``--qps`` / ``--burst``, the chart's defaults unless given):
from the schedules it parses it finds the busiest minute of the next day and warns when that
minute's fires x :data:`REQUESTS_PER_FIRE` exceed a minute of ``--qps`` -- ticks then
collapse and runs are lost without an error (the reference's catch-up runs only the last
missed tick, ``internal/controller/cron_controller.go:408-436``) -- or already past
:data:`TICK_WORK_WARN_FRAC` of it (one slow tick from that cliff), or when its fires exceed
``--burst`` (the last CREATEs land (fires - burst) / qps seconds after the tick).  An upgrade
that keeps the reference's ``qps: 30`` (``/root/reference/cmd/operator/start.go:218-219``)
collapses ticks from about 450 minutely Crons.
"""
from __future__ import annotations

import argparse
import sys
from dataclasses import dataclass, field
from typing import TYPE_CHECKING, Any, Dict, List, Optional, Tuple

from ..api.meta import GroupVersionKind, GroupVersionResource

# the operator's runtime is imported when the check runs, not when the CLI builds its parser
if TYPE_CHECKING:
    from ..runtime.client import Client

# what the reconciler does with a template's kind: LIST/WATCH it (informer), CREATE it on a tick,
# DELETE it (history GC, Replace), GET it (deduplication after a lost response)
NEEDED_VERBS = ("get", "list", "watch", "create", "delete")
LEASES = GroupVersionResource("coordination.k8s.io", "v1", "leases")
# API requests per Cron fire in the default mode: the CREATE, the status PATCH recording it, the
# status PATCH moving the finished job to history, the history-GC DELETE (bench.py
# api_requests_per_fire / deployment_api_requests_per_fire, realistic job lifecycle: 4.0)
REQUESTS_PER_FIRE = 4.0
HORIZON_MINUTES = 24 * 60  # the busiest minute is looked for over the next day
# warn before the cliff: the busiest minute's tick work (its fires' requests at --qps) may take at
# most this share of the minute.  Measured at chart defaults (qps 150 / burst 300, TLS + the etcd
# latency model, realistic job lifecycle): 1000 minutely Crons take 28.7 s of each 60 s tick, p50
# tick->create 1.35 s; 2000 take 57.4 s, p50 4.7 s -- one slow tick from collapse
# (profiles/chart_defaults_mi355x_box_r5.json; docs/benchmarks.md "the chart as installed")
TICK_WORK_WARN_FRAC = 0.8


@dataclass
class KindReport:
    gvk: GroupVersionKind
    crons: List[str] = field(default_factory=list)
    resource: str = ""
    served: bool = False
    missing_verbs: List[str] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return self.served and not self.missing_verbs


@dataclass
class Report:
    crons: int = 0
    kinds: Dict[GroupVersionKind, KindReport] = field(default_factory=dict)
    bad_schedules: List[Tuple[str, str, str]] = field(default_factory=list)   # (cron, schedule, error)
    bad_templates: List[Tuple[str, str]] = field(default_factory=list)        # (cron, error)
    named_templates: List[str] = field(default_factory=list)                  # run as Forbid
    lease: Optional[Dict[str, Any]] = None
    errors: List[str] = field(default_factory=list)
    # client budget: the busiest minute's fires (and when), and the warnings it raises
    peak_fires_per_minute: int = 0
    peak_minute: str = ""
    budget_warnings: List[str] = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return not (self.errors or self.bad_schedules or self.bad_templates or
                    any(not k.ok for k in self.kinds.values()))


def _lease_name() -> str:
    from ..runtime.manager import DEFAULT_LEADER_ELECTION_ID

    return DEFAULT_LEADER_ELECTION_ID


def rbac_missing(group: str, resource: str, rules: List[Dict[str, Any]]) -> List[str]:
    """Verbs of :data:`NEEDED_VERBS` none of ``rules`` grants on ``group/resource``."""
    from ..apiserver.rbac import rule_allows

    return [v for v in NEEDED_VERBS
            if not any(rule_allows(r, {"verb": v, "group": group, "resource": resource, "namespace": "x"})
                       for r in rules)]


def peak_fires(schedules: List[Any], now: Any, engine: Any = None,
               horizon_minutes: int = HORIZON_MINUTES) -> Tuple[int, Any]:
    """(most fires in one minute over the next ``horizon_minutes``, that minute's start).  A
    schedule fires at most once a minute (seconds are fixed at 0), so each contributes at
    most ``horizon_minutes`` ticks.

    ``schedules``: parsed schedules, or ``(schedule, how many Crons use it)`` pairs.  A fleet
    shares a few schedule strings, so each distinct one is walked once and its ticks counted
    with its multiplicity (10,000 Crons of 3 schedules: ~4,300 ``next`` calls, not 14 million)."""
    from collections import Counter

    from ..cron.engine import default_engine
    from ..utils.gotime import GoTime

    eng = engine or default_engine()
    end = now.sec + horizon_minutes * 60
    per_minute: Counter = Counter()
    for item in schedules:
        sched, mult = item if isinstance(item, tuple) else (item, 1)
        t = now
        for _ in range(horizon_minutes + 1):
            t = eng.next(sched, t)
            if t.is_zero() or t.sec > end:
                break
            per_minute[t.sec // 60] += mult
    if not per_minute:
        return 0, None
    minute, n = max(per_minute.items(), key=lambda kv: (kv[1], -kv[0]))
    return n, GoTime(minute * 60, 0, now.loc)


def budget_warnings(fires: int, qps: float, burst: int, requests_per_fire: float = REQUESTS_PER_FIRE) -> List[str]:
    """Warnings for a minute with ``fires`` Cron fires under a ``qps`` / ``burst`` client."""
    out = []
    if qps <= 0 or fires <= 0:
        return out
    need = fires * requests_per_fire / 60.0
    if need > qps:
        out.append(f"the busiest minute has {fires} fires x {requests_per_fire:g} API requests = {need:.0f} QPS, "
                   f"more than --qps {qps:g}: ticks collapse and scheduled runs are lost; set qps >= "
                   f"{need:.0f} (helm: qps), or shard the fleet (sharding.count)")
    elif need > TICK_WORK_WARN_FRAC * qps:
        work = fires * requests_per_fire / qps
        out.append(f"the busiest minute's {fires} fires need about {work:.0f} s of the 60 s minute at --qps "
                   f"{qps:g} ({100 * work / 60:.0f}%, over {100 * TICK_WORK_WARN_FRAC:.0f}%): one slow tick "
                   f"from collapse (measured: 2000 minutely Crons at the chart's defaults take 57.4 s per "
                   f"tick); set qps >= {need / TICK_WORK_WARN_FRAC:.0f} (helm: qps), or shard the fleet "
                   f"(sharding.count)")
    if fires > burst:
        # the tick's first `burst` CREATEs go out at once, the rest at qps (the tick reserve keeps
        # the whole burst for them)
        p50 = max(0.0, fires / 2 - burst) / qps
        out.append(f"the busiest minute's {fires} CREATEs exceed --burst {burst}: the median lands about "
                   f"{p50:.1f} s and the last about {(fires - burst) / qps:.1f} s after the tick (raise burst "
                   f"to {fires} for all at once)")
    return out


async def preflight(client: "Client", namespace: str = "", rules: Optional[List[Dict[str, Any]]] = None,
                    lease_namespace: str = "", qps: float = 0.0, burst: int = 0, now: Any = None) -> Report:
    """Read-only checks of the Crons in ``namespace`` ("" = all) against ``rules`` (default: the
    operator's own RBAC)."""
    from ..api import errors
    from ..api.v1alpha1 import CRON_GVR
    from ..controller.rbac import RULES
    from ..cron.parser import CronParseError, parse_standard
    from ..models.workload import WorkloadError, get_workload_gvk
    from ..runtime.client import NoKindMatchError

    rules = list(RULES) if rules is None else rules
    rep = Report()
    try:
        crons = (await client.list(CRON_GVR, namespace)).get("items") or []
    except errors.ApiError as e:
        rep.errors.append(f"cannot list crons.apps.kubedl.io: {e}")
        return rep
    rep.crons = len(crons)
    from ..cron.engine import ScheduleError, default_engine
    from ..utils.gotime import LOCAL, parse_rfc3339

    engine = default_engine()
    if now is None:
        from ..utils.clock import RealClock

        now = RealClock().now(LOCAL)
    from collections import Counter

    sched_counts: Counter = Counter()  # schedule string -> Crons that fire on it
    for c in crons:
        m = c.get("metadata") or {}
        key = f"{m.get('namespace', '')}/{m.get('name', '')}"
        spec = c.get("spec") or {}
        sched = spec.get("schedule", "")
        try:
            parse_standard(sched)
        except (CronParseError, ValueError) as e:
            rep.bad_schedules.append((key, sched, str(e)))
        else:
            deadline = spec.get("deadline")
            past = False
            if isinstance(deadline, str) and deadline:
                try:
                    past = now.after(parse_rfc3339(deadline))
                except ValueError:
                    past = False
            if not spec.get("suspend") and not past:
                sched_counts[sched] += 1
        wl = (spec.get("template") or {}).get("workload")
        try:
            gvk = get_workload_gvk(wl)
        except WorkloadError as e:
            rep.bad_templates.append((key, str(e)))
            continue
        if isinstance(wl, dict) and (wl.get("metadata") or {}).get("name"):
            rep.named_templates.append(key)
        rep.kinds.setdefault(gvk, KindReport(gvk)).crons.append(key)
    for gvk, kr in rep.kinds.items():
        try:
            gvr, _ = await client.mapper.resource_for(gvk)
        except NoKindMatchError:
            continue
        except errors.ApiError as e:  # discovery itself failed (403, 5xx): say so, do not guess
            rep.errors.append(f"cannot discover {gvk.group}/{gvk.version}: {e}")
            kr.served = True  # unknown, reported as an error above rather than as "not served"
            kr.resource = "?"
            continue
        kr.served, kr.resource = True, gvr.resource
        kr.missing_verbs = rbac_missing(gvk.group, gvr.resource, rules)
    scheds: List[Tuple[Any, int]] = []
    for sched, n in sched_counts.items():  # each distinct schedule (its CRON_TZ= included) once
        try:
            scheds.append((engine.parse(sched), n))
        except ScheduleError:
            pass
    if qps > 0 and scheds:
        rep.peak_fires_per_minute, peak = peak_fires(scheds, now, engine)
        rep.peak_minute = peak.rfc3339() if peak is not None else ""
        rep.budget_warnings = budget_warnings(rep.peak_fires_per_minute, qps, burst)
    if lease_namespace:
        try:
            lease = await client.get(LEASES, lease_namespace, _lease_name())
            rep.lease = lease.get("spec") or {}
        except errors.ApiError as e:
            if e.code != 404:
                rep.errors.append(f"cannot read Lease {lease_namespace}/{_lease_name()}: {e}")
    return rep


def render(rep: Report, lease_namespace: str = "") -> str:
    out = [f"Crons: {rep.crons}"]
    if rep.kinds:
        out.append("")
        out.append(f"{'KIND':<40} {'RESOURCE':<28} {'CRONS':>5}  {'SERVED':<6}  RBAC")
        for gvk, kr in sorted(rep.kinds.items(), key=lambda x: (x[0].group, x[0].kind)):
            kind = f"{gvk.kind}.{gvk.group or 'core'}/{gvk.version}"
            rbac = "ok" if not kr.missing_verbs else "missing " + ",".join(kr.missing_verbs)
            out.append(f"{kind:<40} {kr.resource or '-':<28} {len(kr.crons):>5}  {'yes' if kr.served else 'NO':<6}  "
                       f"{rbac if kr.served else '-'}")
    for key, sched, err in rep.bad_schedules:
        out.append(f"error: {key}: schedule {sched!r} does not parse: {err}")
    for key, err in rep.bad_templates:
        out.append(f"error: {key}: {err}")
    for gvk, kr in rep.kinds.items():
        if not kr.served:
            out.append(f"error: {gvk.kind}.{gvk.group} is not served by this cluster; "
                       f"{len(kr.crons)} Cron(s) would fail to create it: {', '.join(kr.crons[:5])}")
        elif kr.missing_verbs:
            out.append(f"error: the operator's RBAC lacks {','.join(kr.missing_verbs)} on "
                       f"{kr.resource}.{gvk.group}; add it to rbac.extraWorkloadRules")
    for key in rep.named_templates:
        out.append(f"note: {key}: the template sets metadata.name, so the Cron runs as Forbid (OverridePolicy)")
    if rep.peak_fires_per_minute:
        out.append(f"busiest minute (next {HORIZON_MINUTES // 60} h): {rep.peak_fires_per_minute} fires at "
                   f"{rep.peak_minute}")
    for w in rep.budget_warnings:
        out.append(f"warning: {w}")
    if lease_namespace:
        if rep.lease:
            out.append(f"lease {lease_namespace}/{_lease_name()}: held by "
                       f"{rep.lease.get('holderIdentity', '?')}, renewed {rep.lease.get('renewTime', '?')}, "
                       f"duration {rep.lease.get('leaseDurationSeconds', '?')} s")
        else:
            out.append(f"lease {lease_namespace}/{_lease_name()}: none (no operator is leading)")
    out.extend(f"error: {e}" for e in rep.errors)
    out.append("preflight: ok" if rep.ok else "preflight: FAILED")
    return "\n".join(out) + "\n"


def add_parser(sub: Any) -> None:
    pf = sub.add_parser("preflight", help="Check a cluster's Crons before this operator takes it over "
                                          "(read-only)")
    pf.add_argument("--kubeconfig", default="")
    pf.add_argument("-n", "--namespace", default="", help="only this namespace (default: all)")
    pf.add_argument("--lease-namespace", default="",
                    help="also report the holder of the leader Lease in this namespace")
    pf.add_argument("--extra-rules", default="",
                    help="YAML list of {apiGroups, resources} rules, as the chart's rbac.extraWorkloadRules")
    from .main import DEFAULT_BURST, DEFAULT_QPS

    pf.add_argument("--qps", type=float, default=DEFAULT_QPS,
                    help="the operator's --qps to size against (helm: qps; the reference ships 30)")
    pf.add_argument("--burst", type=int, default=DEFAULT_BURST,
                    help="the operator's --burst to size against (helm: burst; the reference ships 50)")


async def run(a: argparse.Namespace) -> int:
    import yaml

    from ..controller.rbac import RULES
    from ..runtime.client import Client
    from ..runtime.http import HttpTransport
    from ..runtime.kubeconfig import ConfigError, get_config

    try:
        cfg = get_config(a.kubeconfig)
    except ConfigError as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    rules = list(RULES)
    if a.extra_rules:
        with open(a.extra_rules) as fh:
            for r in yaml.safe_load(fh) or []:
                rules.append({"apiGroups": r.get("apiGroups") or [], "resources": r.get("resources") or [],
                              "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]})
    client = Client(HttpTransport(cfg), qps=-1)
    try:
        rep = await preflight(client, a.namespace, rules, a.lease_namespace, qps=a.qps, burst=a.burst)
    finally:
        await client.close()
    sys.stdout.write(render(rep, a.lease_namespace))
    return 0 if rep.ok else 1
