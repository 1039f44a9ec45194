"""Controller wiring -- ``SetupWithManager`` (``internal/controller/cron_controller.go:69-77``).

* ``For(&Cron{})`` -- the Cron informer feeds the queue; with
  ``own_write_filter`` the update events produced by our own status patches
  are dropped (the reconcile they would trigger recomputes the same status);
* ``Owns(PyTorchJob)``, ``Owns(TFJob)`` -- as in the reference; the informers are
  label-selected on ``kubedl.io/cron-name`` in cache mode (we only ever need
  children), unfiltered in reference/live mode;
* with ``dynamic_watches`` any other template kind (MPIJob, batch Job, Pod, ...)
  gets an owned watch the first time a Cron uses it, so its completion is
  noticed (the reference never watches MPIJob);
* ``WithLogConstructor(logConstructor(..., "cron"))`` (``util.go:27-41``).

RBAC (the reference's markers at ``cron_controller.go:79-85`` name the wrong
group ``kubedl.io``) is generated with the correct group
by :mod:`cron_operator_amd.controller.rbac`.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

from ..api import errors
from ..api.meta import GroupVersionKind
from ..api.v1alpha1 import CRON_GVK, LABEL_CRON_NAME
from ..cron.engine import CronEngine
from ..models.workload import WorkloadPolicy, classify
from ..runtime.controller import Controller
from ..runtime.informer import EventHandler, Informer, label_index, strip_managed_fields
from ..runtime.manager import Manager
from ..utils.logging import get_logger, log_constructor
from . import sharding
from .reconciler import CHILD_INDEX, CronReconciler, ReconcilerOptions, WireCodecs

CONTROLLER_NAME = "cron"

# child metadata a reconcile reads: identity, the cron-name label and owner (which Cron lists it),
# creation time (history order), deletion
_CHILD_META = ("name", "namespace", "uid", "labels", "ownerReferences", "creationTimestamp",
               "deletionTimestamp")


def child_update_matters(old, new, gvk: GroupVersionKind, policy: WorkloadPolicy, new_info=None) -> bool:
    """Can this child update change its Cron's reconcile?  Not when the child stays running and
    nothing a reconcile reads moved: its active ref keeps the resourceVersion it entered
    ``status.active`` with (``active_ref_resource_version="first"``), and an unfinished child's
    status feeds nothing else.  The training-operator's Created / replicaStatuses / Running
    writes are such updates (``/root/reference/test/crds/kubeflow.org_pytorchjobs.yaml:4739-4828``);
    the reference requeues the Cron on each (``cron_controller.go:70-77``, no predicates)."""
    om, nm = old.get("metadata") or {}, new.get("metadata") or {}
    if om is not nm and [*map(om.get, _CHILD_META)] != [*map(nm.get, _CHILD_META)]:  # compared in C
        return True
    try:
        # ``new_info``: the child informer's memo of ``new`` (child_info), computed already
        if new_info is not None and new_info.obj is new:
            if new_info.err is not None or new_info.finished:
                return True
        elif classify(new, gvk, policy).finished:
            return True
        return classify(old, gvk, policy).finished
    except Exception:  # noqa: BLE001 - an unreadable status: let the reconcile report it
        return True


async def setup_with_manager(mgr: Manager, options: Optional[ReconcilerOptions] = None,
                             engine: Optional[CronEngine] = None) -> Tuple[Controller, CronReconciler]:
    opts = options or ReconcilerOptions()
    log = get_logger()
    index, count = mgr.opts.shard_index, mgr.opts.shard_count
    if mgr.opts.shard_routing not in sharding.ROUTINGS:
        raise ValueError(f"unknown shard routing {mgr.opts.shard_routing!r}")
    by_label = count > 1 and mgr.opts.shard_routing == "labels"
    by_hash = count > 1 and not by_label
    codecs = WireCodecs(opts.slim_child_cache, compact_metadata=opts.compact_metadata(),
                        shard=(index, count) if by_hash else None) if opts.wire_codecs else None
    cron_inf = await mgr.cache.get_informer(CRON_GVK,
                                            label_selector=sharding.shard_selector(index, count) if by_label else None,
                                            transform=strip_managed_fields if opts.slim_child_cache else None,
                                            decoder=codecs.cron_event if codecs is not None else None,
                                            list_decoder=codecs.cron_list if codecs is not None else None,
                                            keep=sharding.hash_keep(index, count, False) if by_hash else None)
    rec = CronReconciler(mgr.client, mgr.cache, mgr.get_event_recorder_for(CONTROLLER_NAME), mgr.clock, engine,
                         opts, cron_inf, codecs)
    if codecs is not None:
        mgr.add_debug_view("wire-memo", codecs.memo.stats)
    ctrl = Controller(CONTROLLER_NAME, rec, mgr.clock, mgr.opts.max_concurrent_reconciles, log)
    ctrl.set_log_constructor(log_constructor(log, "Cron"))
    assigner: Optional[sharding.ShardAssigner] = None
    if count > 1:
        ctrl.set_shard(index, count)  # with label routing too: a mislabelled object is never reconciled twice
    if by_hash:
        rec.child_keep = sharding.hash_keep(index, count, True)
    if by_label:
        rec.child_selector = sharding.child_selector(index, count)
        rec.child_labels = {sharding.LABEL_SHARD: sharding.shard_label_value(index, count)}
        assigner = sharding.ShardAssigner(mgr.client, index, count)
        await assigner.watch(mgr.cache, CRON_GVK, child=False)
        mgr.add(assigner.run)
    rec.shard_assigner = assigner
    if assigner is not None and opts.list_mode == "cache":
        # a Cron joins this shard only once its relabelled children are in this shard's child
        # informers.  A kind with no informer yet is not waited for: the first reconcile that
        # needs it starts the informer and waits for its LIST, which holds the child.  Live mode
        # (--compat-mode reference) LISTs children from the apiserver: nothing to wait for.
        def observed(gvk: GroupVersionKind, ns: str, name: str) -> bool:
            inf = rec.child_informers.get(gvk)
            return inf is None or inf.get(ns, name, copy=False) is not None
        assigner.observed = observed

    preds = []
    if opts.own_write_filter:
        def not_own_write(event: str, old, new) -> bool:
            return not (event == "update" and rec.is_own_write(old, new))
        preds.append(not_own_write)
    ctrl.watch_for(cron_inf, CRON_GVK, preds)

    watched: Dict[GroupVersionKind, Informer] = {}

    def attach(gvk: GroupVersionKind, inf: Informer) -> None:
        if gvk in watched:
            return
        watched[gvk] = inf

        def key_of(obj) -> str:
            m = obj.get("metadata") or {}
            return f"{m.get('namespace', '')}/{(m.get('labels') or {}).get(LABEL_CRON_NAME, '')}"

        # one predicate for the child events (no per-event loop over several): creates and deletes
        # that only confirm what the reconciler already folded into status are dropped, and so are
        # updates that change nothing a reconcile reads
        # (an expected event is only redundant when the reconciler folded its own CREATE / DELETE
        # into status.active itself)
        skip_expected = opts.expectations and opts.skip_expected_events and opts.fold_created_into_active
        skip_unchanged = opts.skip_unchanged_child_updates and opts.active_ref_resource_version != "live"
        policy = opts.workload
        ex = rec.expect

        def owned_event(event: str, old, new, g=gvk, i=inf) -> bool:
            if event == "update":
                if not skip_unchanged or old is None:
                    return True
                m = new.get("metadata") or {}
                return child_update_matters(old, new, g, policy,
                                            i.derived.get(f"{m.get('namespace', '')}/{m.get('name', '')}"))
            if not skip_expected:
                return True
            if event == "create":
                return not (ex.pending or ex.created) or not ex.matches_created(key_of(new), new)
            if event == "delete":
                return not ex.deleted or not ex.matches_deleted(key_of(new), new)
            return True
        ctrl.watch_owned(inf, CRON_GVK, [owned_event] if skip_expected or skip_unchanged else [])
        if assigner is not None:
            assigner.watch_soon(mgr.cache, gvk, child=True)
        if opts.expectations:
            exp = rec.expect

            # most events find no expectation at all: skip building the key then
            def observe_add(o) -> None:
                if exp.created:
                    exp.observe_add(key_of(o), (o.get("metadata") or {}).get("uid", ""))
                if exp.pending:  # a CREATE whose response never came (cancelled): the job is here
                    exp.drop_pending(key_of(o), (o.get("metadata") or {}).get("name", ""))

            def observe_delete(o) -> None:
                if exp.created or exp.deleted:
                    exp.observe_delete(key_of(o), (o.get("metadata") or {}).get("uid", ""))

            inf.add_handler(EventHandler(on_add=observe_add, on_update=lambda old, o: observe_add(o),
                                         on_delete=observe_delete))
        if opts.classification_cache:
            inf.add_handler(EventHandler(
                on_delete=lambda o: rec.forget_child((o.get("metadata") or {}).get("uid", ""))))

    for gvk in opts.static_owned_kinds:
        try:
            if opts.list_mode == "cache":
                inf = await mgr.cache.get_informer(gvk, label_selector=rec.child_selector,
                                                   indexers={CHILD_INDEX: label_index(LABEL_CRON_NAME)},
                                                   transform=rec.child_transform(gvk),
                                                   decoder=codecs.child_event if codecs is not None else None,
                                                   list_decoder=codecs.child_list if codecs is not None else None,
                                                   keep=rec.child_keep)
                rec.child_informers[gvk] = inf
                rec.ensure_derive(inf, gvk)
            else:
                inf = await mgr.cache.get_informer(gvk, label_selector=rec.child_selector if by_label else None,
                                                   keep=rec.child_keep)
            if assigner is not None:
                await assigner.watch(mgr.cache, gvk, child=True)
        except errors.ApiError as e:
            # the reference fails to start without these CRDs; we keep running and
            # pick the kind up lazily once a Cron uses it
            log.info("owned kind not served by the apiserver, watching lazily", kind=gvk.kind, error=str(e))
            continue
        attach(gvk, inf)

    if opts.dynamic_watches:
        rec.on_child_informer = attach
    mgr.add_controller(ctrl)
    return ctrl, rec
