"""Prometheus metrics with controller-runtime / client-go / workqueue names.

The reference registers no custom collectors; it exposes controller-runtime's
defaults on ``/metrics`` (the e2e TODO at ``test/e2e/e2e_test.go:281-289``
targets ``controller_runtime_reconcile_total``).  The same series exist here so
dashboards and alerts carry over:

* ``controller_runtime_reconcile_total{controller,result}``,
  ``..._reconcile_errors_total``, ``..._terminal_reconcile_errors_total``,
  ``..._reconcile_panics_total``, ``..._reconcile_time_seconds``,
  ``..._max_concurrent_reconciles``, ``..._active_workers``;
* ``workqueue_{depth,adds_total,queue_duration_seconds,work_duration_seconds,
  unfinished_work_seconds,longest_running_processor_seconds,retries_total}``;
* ``rest_client_requests_total{code,host,method}``,
  ``rest_client_request_duration_seconds``, ``rest_client_rate_limiter_duration_seconds``;
* ``leader_election_master_status{name}``;
* ``certwatcher_read_certificate_total`` / ``..._errors_total`` (a ``--metrics-cert-path``
  certificate is reloaded when rotated);
* process and Python runtime collectors (the Go/process collectors' counterpart).

The series live in :mod:`cron_operator_amd.runtime.promlite`, a small client
whose per-update cost is an attribute add (the operator is one asyncio thread).

Operator-specific additions (``cron_operator_*``): tick->create latency,
workloads created/deleted, missed ticks and status patches.
"""
from __future__ import annotations

from .promlite import Counter, Gauge, Histogram, ObservedGauge, ProcessCollector, PythonCollector, Registry

REGISTRY = Registry()
ProcessCollector(registry=REGISTRY)
PythonCollector(registry=REGISTRY)

_RECONCILE_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.15, 0.2, 0.25, 0.3, 0.35, 0.4, 0.45, 0.5, 0.6, 0.7, 0.8,
                      0.9, 1.0, 1.25, 1.5, 1.75, 2.0, 2.5, 3.0, 3.5, 4.0, 4.5, 5, 6, 7, 8, 9, 10, 15, 20, 25, 30,
                      40, 50, 60)
_WQ_BUCKETS = tuple(10.0 ** e for e in range(-8, 4))

RECONCILE_TOTAL = Counter("controller_runtime_reconcile_total", "Total number of reconciliations per controller",
                          ["controller", "result"], registry=REGISTRY)
RECONCILE_ERRORS = Counter("controller_runtime_reconcile_errors_total",
                           "Total number of reconciliation errors per controller", ["controller"], registry=REGISTRY)
TERMINAL_ERRORS = Counter("controller_runtime_terminal_reconcile_errors_total",
                          "Total number of terminal reconciliation errors per controller", ["controller"],
                          registry=REGISTRY)
RECONCILE_PANICS = Counter("controller_runtime_reconcile_panics_total",
                           "Total number of reconciliation panics per controller", ["controller"], registry=REGISTRY)
RECONCILE_TIME = Histogram("controller_runtime_reconcile_time_seconds",
                           "Length of time per reconciliation per controller", ["controller"],
                           buckets=_RECONCILE_BUCKETS, registry=REGISTRY)
MAX_CONCURRENT = Gauge("controller_runtime_max_concurrent_reconciles",
                       "Maximum number of concurrent reconciles per controller", ["controller"], registry=REGISTRY)
ACTIVE_WORKERS = Gauge("controller_runtime_active_workers",
                       "Number of currently used workers per controller", ["controller"], registry=REGISTRY)

WQ_DEPTH = Gauge("workqueue_depth", "Current depth of workqueue", ["name", "controller"], registry=REGISTRY)
WQ_ADDS = Counter("workqueue_adds_total", "Total number of adds handled by workqueue", ["name", "controller"],
                  registry=REGISTRY)
WQ_LATENCY = Histogram("workqueue_queue_duration_seconds",
                       "How long in seconds an item stays in workqueue before being requested",
                       ["name", "controller"], buckets=_WQ_BUCKETS, registry=REGISTRY)
WQ_WORK = Histogram("workqueue_work_duration_seconds", "How long in seconds processing an item from workqueue takes.",
                    ["name", "controller"], buckets=_WQ_BUCKETS, registry=REGISTRY)
WQ_UNFINISHED = Gauge("workqueue_unfinished_work_seconds",
                      "How many seconds of work has been done that is in progress and hasn't been observed by "
                      "work_duration.", ["name", "controller"], registry=REGISTRY)
WQ_LONGEST = Gauge("workqueue_longest_running_processor_seconds",
                   "How many seconds has the longest running processor for workqueue been running.",
                   ["name", "controller"], registry=REGISTRY)
WQ_RETRIES = Counter("workqueue_retries_total", "Total number of retries handled by workqueue",
                     ["name", "controller"], registry=REGISTRY)

REST_REQUESTS = Counter("rest_client_requests_total",
                        "Number of HTTP requests, partitioned by status code, method, and host.",
                        ["code", "host", "method"], registry=REGISTRY)
REST_RETRIES = Counter("rest_client_request_retries_total",
                       "Number of request retries, partitioned by status code, verb, and host.",
                       ["code", "verb", "host"], registry=REGISTRY)
REST_LATENCY = Histogram("rest_client_request_duration_seconds", "Request latency in seconds. Broken down by verb, "
                         "and host.", ["verb", "host"],
                         buckets=(0.005, 0.025, 0.1, 0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 15.0, 30.0, 60.0),
                         registry=REGISTRY)
REST_RATE_LIMIT = Histogram("rest_client_rate_limiter_duration_seconds",
                            "Client side rate limiter latency in seconds. Broken down by verb, and host.",
                            ["verb", "host"], buckets=(0.005, 0.025, 0.1, 0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 15.0, 30.0,
                                                       60.0), registry=REGISTRY)

LEADER_STATUS = Gauge("leader_election_master_status",
                      "Gauge of if the reporting system is master of the relevant lease, 0 indicates backup, 1 "
                      "indicates master. 'name' is the string used to identify the lease.", ["name"],
                      registry=REGISTRY)

SCHEDULE_LATENCY = Histogram("cron_operator_schedule_latency_seconds",
                             "Delay between a scheduled tick and the CREATE of its workload.", ["controller"],
                             buckets=(0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120,
                                      300), registry=REGISTRY)
WORKLOADS_CREATED = Counter("cron_operator_workloads_created_total", "Workloads created by Crons.", ["kind"],
                            registry=REGISTRY)
WORKLOADS_DELETED = Counter("cron_operator_workloads_deleted_total", "Workloads deleted by Crons.",
                            ["kind", "reason"], registry=REGISTRY)
MISSED_TICKS = Counter("cron_operator_missed_ticks_total", "Scheduled ticks collapsed into a later run.",
                       registry=REGISTRY)
STATUS_PATCHES = Counter("cron_operator_status_patches_total", "Cron status writes.", ["result"], registry=REGISTRY)
# released worker slots (runtime/controller.py release_worker) and the client's request gates
# (runtime/ratelimit.py), read at scrape time
RECONCILES_WRITING = ObservedGauge("cron_operator_reconciles_writing",
                                   "Reconciles that released their worker slot and are finishing their API writes.",
                                   ["controller"], registry=REGISTRY)
WORKER_RELEASES = ObservedGauge("cron_operator_worker_releases_total",
                                "Reconciles that released their worker slot once only API writes were left.",
                                ["controller"], kind="counter", registry=REGISTRY)
REST_INFLIGHT = ObservedGauge("rest_client_requests_in_flight", "API requests in flight (watches excluded).",
                              ["host"], registry=REGISTRY)
REST_WAITING = ObservedGauge("rest_client_requests_waiting",
                             "API requests waiting on the client's QPS bucket or in-flight cap, by priority.",
                             ["host", "gate", "priority"], registry=REGISTRY)


_CHILDREN: dict = {}


def child(metric, *labels: str):
    """``metric.labels(*labels)`` memoised: the reconcile hot path resolves the same few
    label sets over and over."""
    key = (id(metric), labels)
    c = _CHILDREN.get(key)
    if c is None:
        c = _CHILDREN[key] = metric.labels(*labels)
    return c


def exposition() -> bytes:
    return REGISTRY.exposition()

CERT_READS = Counter("certwatcher_read_certificate_total", "Total number of certificate reads", registry=REGISTRY)
CERT_READ_ERRORS = Counter("certwatcher_read_certificate_errors_total", "Total number of certificate read errors",
                           registry=REGISTRY)
