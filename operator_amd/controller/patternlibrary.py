"""PatternLibrary reconciler (J/reconcile/PatternLibraryReconciler.java:49-103).

* gate on the refresh interval: no sync if ``now <= lastSyncTime + interval``
  (:60-65, :207-245) — we return "no update, reschedule at the due time";
* phase Syncing -> per-repository sync (failures recorded, never fatal: :114-134)
  -> availableLibraries -> phase Ready "Sync completed: %d repositories,
  %d libraries available" (:85-91) -> reschedule after the interval (:94-95);
  an exception -> phase Failed "Failed to reconcile: <msg>" (:97-101);
* refresh interval grammar: ``Ns | Nm | Nh | Nd | NhMm`` (case-insensitive,
  trimmed), anything else -> 1 hour (:282-306);
* fixes: credentials are read from the PatternLibrary's own
  namespace (falling back to ``podmortem-system``), the ``token`` key (or
  ``username`` + ``password``) is base64-DECODED; ``syncedRepositories`` is
  populated {name, lastCommit, syncTime, status, error}.
After a successful sync the ``on_synced`` hook recompiles the pattern set.
"""
from __future__ import annotations

import base64
import datetime as dt
import logging
import re
from typing import Callable

from operator_amd.kube.resources import PATTERNLIBRARIES, SECRETS, ApiError
from operator_amd.utils.timefmt import instant_str, now, parse_instant

from .runtime import UpdateControl
from .sync import PatternSync

log = logging.getLogger(__name__)

DEFAULT_INTERVAL_S = 3600
LEGACY_SECRET_NAMESPACE = "podmortem-system"


def parse_refresh_interval(value: str | None) -> dt.timedelta:
    v = (value or "").strip().lower() or "1h"
    m = re.fullmatch(r"(\d+)([smhd])", v)
    if m:
        n = int(m.group(1))
        return {"s": dt.timedelta(seconds=n), "m": dt.timedelta(minutes=n), "h": dt.timedelta(hours=n),
                "d": dt.timedelta(days=n)}[m.group(2)]
    m = re.fullmatch(r"(\d+)h(\d+)m", v)
    if m:
        return dt.timedelta(hours=int(m.group(1)), minutes=int(m.group(2)))
    log.warning("Unrecognized refresh interval format: '%s', defaulting to 1 hour", v)
    return dt.timedelta(hours=1)


def needs_sync(lib: dict, at: dt.datetime | None = None) -> bool:
    st = lib.get("status") or {}
    last = parse_instant(st.get("lastSyncTime"))
    if last is None:
        return True
    interval = parse_refresh_interval((lib.get("spec") or {}).get("refreshInterval"))
    return (at or now()) > last + interval


class PatternLibraryReconciler:
    def __init__(self, kube, sync: PatternSync, on_synced: Callable[[dict], None] | None = None, clock=now):
        self.kube, self.sync = kube, sync
        self.on_synced = on_synced
        self.clock = clock

    def credentials(self, lib: dict, secret_ref: str) -> str | None:
        ns = (lib.get("metadata") or {}).get("namespace")
        for n in dict.fromkeys([ns, LEGACY_SECRET_NAMESPACE]):
            if not n:
                continue
            try:
                sec = self.kube.get(SECRETS, secret_ref, n)
            except ApiError as e:
                log.warning("Failed to get credentials from secret %s: %s", secret_ref, e)
                continue
            if sec is None or not sec.get("data"):
                continue
            data = sec["data"]

            def dec(k):
                return base64.b64decode(data[k]).decode("utf-8", "replace")

            try:
                if "token" in data:
                    return dec("token")
                if "username" in data and "password" in data:
                    return f"{dec('username')}:{dec('password')}"
            except Exception as e:  # noqa: BLE001
                log.warning("Secret %s/%s is not valid base64: %s", n, secret_ref, e)
        return None

    def reconcile(self, lib: dict) -> UpdateControl:
        md = lib.get("metadata") or {}
        name = md.get("name")
        spec = lib.get("spec") or {}
        interval = parse_refresh_interval(spec.get("refreshInterval"))
        t = self.clock()
        if not needs_sync(lib, t):
            last = parse_instant((lib.get("status") or {}).get("lastSyncTime"))
            due = max(1.0, ((last + interval) - t).total_seconds()) if last else interval.total_seconds()
            return UpdateControl.no_update(reschedule_after=due)
        try:
            self.kube.patch_status(PATTERNLIBRARIES, name, md.get("namespace"),
                                   {"phase": "Syncing", "message": "Synchronizing pattern repositories",
                                    "observedGeneration": md.get("generation")})
            repos = spec.get("repositories") or []
            synced = []
            for repo in repos:
                entry = {"name": repo.get("name"), "syncTime": instant_str()}
                try:
                    creds = None
                    secret_ref = (repo.get("credentials") or {}).get("secretRef")
                    if secret_ref:
                        creds = self.credentials(lib, secret_ref)
                    entry["lastCommit"] = self.sync.sync_repository(name, repo, creds)
                    entry["status"] = "Success"
                except Exception as e:  # noqa: BLE001 (per-repo failures are swallowed: :130-133)
                    log.error("Failed to sync repository %s: %s", repo.get("name"), e)
                    entry["status"] = "Failed"
                    entry["error"] = str(e)
                synced.append(entry)
            available = self.sync.available_libraries(name)
            status = {"phase": "Ready",
                      "message": f"Sync completed: {len(repos)} repositories, {len(available)} libraries available",
                      "lastSyncTime": instant_str(), "availableLibraries": available,
                      "syncedRepositories": synced, "observedGeneration": md.get("generation")}
            if self.on_synced is not None:
                try:
                    self.on_synced(lib)
                except Exception as e:  # noqa: BLE001
                    log.error("pattern reload after sync of %s failed: %s", name, e)
            return UpdateControl.patch_status(status, reschedule_after=interval.total_seconds())
        except Exception as e:  # noqa: BLE001
            log.error("Error reconciling PatternLibrary: %s: %s", name, e)
            return UpdateControl.patch_status({"phase": "Failed", "message": f"Failed to reconcile: {e}",
                                               "lastSyncTime": instant_str(),
                                               "observedGeneration": md.get("generation")})

