"""Python-facing wrapper of the native cron engine (``csrc/cron_engine.cpp``).

Zones: the extension knows nothing about the filesystem.  This module hands it
TZif blobs found the way Go's ``time.LoadLocation`` finds them
(:func:`~cron_operator_amd.utils.gotime.tzif_bytes`: ``$ZONEINFO``, the system
zoneinfo directories, then the ``tzdata`` wheel) and maps :class:`~cron_operator_amd.utils.gotime.Location` objects to
native zone ids.  ``Local`` is resolved the same way Go resolves ``time.Local``
($TZ, else /etc/localtime, else UTC).
"""
from __future__ import annotations

import importlib
import os
import threading
from typing import Dict, Optional

from ..utils.gotime import LOCAL, UTC, FixedZone, Location, ZoneLocation, load_location, tzif_bytes
from . import build as _build

_lock = threading.Lock()
_mod = None
_zone_ids: Dict[str, int] = {}
_load_error: Optional[BaseException] = None


def _tzif_bytes(name: str) -> bytes:
    return tzif_bytes(name)


def load(build_if_missing: bool = True):
    """Import (building first if needed) the extension; raises on failure."""
    global _mod, _load_error
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            if build_if_missing and _build.needs_build("_cron_engine"):
                _build.build_extension("_cron_engine")
            mod = importlib.import_module("cron_operator_amd.ops._cron_engine")
            mod.set_zone_resolver(_resolve_name)
            if hasattr(mod, "rfc3339_z"):
                from ..utils import gotime

                gotime.install_native(mod.rfc3339_z, mod.format_rfc3339)
            _mod = mod
        except BaseException as e:  # noqa: BLE001 - recorded for diagnostics
            _load_error = e
            raise
    return _mod


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False



def _resolve_name(name: str) -> int:
    return zone_id(load_location(name))


# the last resolution of Local: (its current implementation object, zone id).  LOCAL.reset()
# (tests changing $TZ) makes impl() return a new object, which misses this cache.
_local_hit: Optional[tuple] = None
# other Locations are immutable: their id is resolved once (the reconciler asks on every
# schedule computation -- several times per Cron fire)
_by_loc: Dict[Location, int] = {}


def zone_id(loc: Location) -> int:
    """Native zone id for a Location (registering it on first use)."""
    global _local_hit
    if loc is UTC:
        return 0
    if loc is LOCAL:
        impl = LOCAL.impl()
        hit = _local_hit
        if hit is not None and hit[0] is impl:
            return hit[1]
        zid = _zone_id_slow(loc)
        _local_hit = (impl, zid)
        return zid
    zid = _by_loc.get(loc)
    if zid is None:
        if len(_by_loc) >= 4096:  # e.g. a FixedZone per parsed "+08:00" timestamp
            _by_loc.clear()
        zid = _by_loc[loc] = _zone_id_slow(loc)
    return zid


def _zone_id_slow(loc: Location) -> int:
    mod = load()
    if loc is LOCAL:
        impl = LOCAL.impl()
        key = "Local:" + (impl.key if isinstance(impl, ZoneLocation) else f"fixed{impl.fixed}")
        zid = _zone_ids.get(key)
        if zid is None:
            if isinstance(impl, ZoneLocation):
                zid = mod.register_zone("Local", _tzif_bytes(impl.key))
            else:
                zid = mod.register_fixed_zone("Local", int(impl.fixed or 0))
            _zone_ids[key] = zid
        return zid
    if isinstance(loc, FixedZone):
        key = f"fixed:{loc.name}:{loc.offset}"
        zid = _zone_ids.get(key)
        if zid is None:
            zid = mod.register_fixed_zone(loc.name, loc.offset)
            _zone_ids[key] = zid
        return zid
    if isinstance(loc, ZoneLocation):
        key = "zone:" + loc.key
        zid = _zone_ids.get(key)
        if zid is None:
            zid = mod.register_zone(loc.name, _tzif_bytes(loc.key))
            _zone_ids[key] = zid
        return zid
    raise TypeError(f"unsupported location {loc!r}")



def engine_path() -> str:
    mod = load()
    return os.path.abspath(mod.__file__)
