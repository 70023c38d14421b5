"""Python reader of the daemon's shared always-on CPU counters
(``dynolog --shared_counters=instructions,cycles``; src/pmu/SharedCounters.h).

The daemon counts once per CPU and publishes cumulative, multiplex-scaled
values in ``/dev/shm/<name>`` under a seqlock; any process reads them without
opening perf events (the reference's BPerf sharing role, BPerfEventsGroup.h).

    r = SharedCounters()           # default segment "dynolog_shared_counters"
    r.rebase(); work(); print(r.delta())   # {"instructions": ..., "cycles": ...}

Per cgroup (``--shared_counters_cgroups=/,/kubepods``; src/pmu/CgroupCounters.h)::

    c = CgroupCounters()           # segment "dynolog_shared_counters_cgroups"
    c.rebase(); work(); print(c.delta("/kubepods"))  # this reader's own offsets
"""
from __future__ import annotations

import mmap
import os
import struct
import time
from typing import Dict, List, Optional

_MAGIC = 0x44594E4F42504552
_MAX_EVENTS = 8
_NAME_LEN = 48
_HDR = struct.Struct("=QIIIIQQQ")          # magic, version, cpus, events, pad, seq, updateNs, publishes
_DATA_OFF = _HDR.size + _MAX_EVENTS * _NAME_LEN


class SharedCounters:
    def __init__(self, name: str = "dynolog_shared_counters"):
        path = "/dev/shm/" + name
        fd = os.open(path, os.O_RDONLY)
        try:
            self._mm = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
        finally:
            os.close(fd)
        magic, _ver, self.num_cpus, self.num_events, _pad, _seq, _u, _p = _HDR.unpack_from(self._mm, 0)
        if magic != _MAGIC:
            raise ValueError(f"{path}: not a dynolog shared-counter segment")
        self.names: List[str] = []
        for i in range(self.num_events):
            raw = self._mm[_HDR.size + i * _NAME_LEN:_HDR.size + (i + 1) * _NAME_LEN]
            self.names.append(raw.split(b"\0", 1)[0].decode())
        self._base: Optional[Dict[str, float]] = None

    def snapshot(self, timeout_s: float = 2.0) -> dict:
        """Consistent per-CPU snapshot (seqlock read).  Retries while the
        writer holds the sequence odd or moved it under the read; a writer
        descheduled mid-update (loaded host) can hold it for a scheduler
        tick, so the bound is time, not a retry count."""
        row = struct.Struct("=" + "d" * (self.num_events + 2))
        deadline = time.monotonic() + timeout_s
        tries = 0
        while True:
            seq0 = struct.unpack_from("=Q", self._mm, 24)[0]
            if not seq0 & 1:
                _, _, _, _, _, _, update_ns, publishes = _HDR.unpack_from(self._mm, 0)
                per_cpu = [list(row.unpack_from(self._mm, _DATA_OFF + c * row.size))[:self.num_events]
                           for c in range(self.num_cpus)]
                if struct.unpack_from("=Q", self._mm, 24)[0] == seq0:
                    return {"update_ns": update_ns, "publishes": publishes, "per_cpu": per_cpu}
            tries += 1
            if time.monotonic() > deadline:
                raise TimeoutError("shared counters: writer kept the seqlock busy")
            time.sleep(0 if tries < 100 else 0.0005)

    def totals(self) -> Dict[str, float]:
        snap = self.snapshot()
        return {n: sum(r[i] for r in snap["per_cpu"]) for i, n in enumerate(self.names)}

    def rebase(self) -> None:
        self._base = self.totals()

    def delta(self) -> Dict[str, float]:
        t = self.totals()
        if self._base is None:
            return t
        return {k: v - self._base.get(k, 0.0) for k, v in t.items()}

    def close(self) -> None:
        self._mm.close()


_CG_MAGIC = 0x44594E4F43475250
_CG_MAX_TARGETS = 64
_CG_PATH_LEN = 192
_CG_HDR = struct.Struct("=QIIIIQQQQ")   # magic, version, events, targets, pad, seq, updateNs, publishes, slices
_CG_DATA_OFF = _CG_HDR.size + _MAX_EVENTS * _NAME_LEN + _CG_MAX_TARGETS * _CG_PATH_LEN


class CgroupCounters:
    """Reader of the per-cgroup segment: cumulative counts of every watched
    cgroup (itself + descendants up to 10 levels) and the system total ("*")."""

    def __init__(self, name: str = "dynolog_shared_counters_cgroups"):
        path = "/dev/shm/" + name
        fd = os.open(path, os.O_RDONLY)
        try:
            self._mm = mmap.mmap(fd, 0, prot=mmap.PROT_READ)
        finally:
            os.close(fd)
        magic, _ver, self.num_events, self.num_targets, *_ = _CG_HDR.unpack_from(self._mm, 0)
        if magic != _CG_MAGIC:
            raise ValueError(f"{path}: not a dynolog cgroup-counter segment")

        def cstr(off, n):
            return self._mm[off:off + n].split(b"\0", 1)[0].decode()
        self.names = [cstr(_CG_HDR.size + i * _NAME_LEN, _NAME_LEN) for i in range(self.num_events)]
        base = _CG_HDR.size + _MAX_EVENTS * _NAME_LEN
        self.paths = [cstr(base + i * _CG_PATH_LEN, _CG_PATH_LEN) for i in range(self.num_targets)]
        self._base: Optional[Dict[str, Dict[str, float]]] = None

    def snapshot(self, timeout_s: float = 2.0) -> dict:
        n = self.num_events
        row = struct.Struct("=" + "d" * n)
        deadline = time.monotonic() + timeout_s
        while True:
            seq0 = struct.unpack_from("=Q", self._mm, 24)[0]
            if not seq0 & 1:
                _, _, _, _, _, _, update_ns, publishes, slices = _CG_HDR.unpack_from(self._mm, 0)
                rows = [row.unpack_from(self._mm, _CG_DATA_OFF + i * row.size) for i in range(1 + self.num_targets)]
                if struct.unpack_from("=Q", self._mm, 24)[0] == seq0:
                    totals = {"*": dict(zip(self.names, rows[0]))}
                    for p, r in zip(self.paths, rows[1:]):
                        totals[p] = dict(zip(self.names, r))
                    return {"update_ns": update_ns, "publishes": publishes, "slices": slices,
                            "totals": totals}
            if time.monotonic() > deadline:
                raise TimeoutError("cgroup counters: writer kept the seqlock busy")
            time.sleep(0.0002)

    def rebase(self) -> None:
        self._base = self.snapshot()["totals"]

    def delta(self, path: str = "*") -> Dict[str, float]:
        cur = self.snapshot()["totals"][path]
        if self._base is None:
            return dict(cur)
        return {k: v - self._base[path].get(k, 0.0) for k, v in cur.items()}

    def close(self) -> None:
        self._mm.close()
