"""Python reader of the daemon's shared always-on CPU counters
(``dynolog --shared_counters=instructions,cycles``; src/pmu/SharedCounters.h).

The daemon counts once per CPU and publishes cumulative, multiplex-scaled
values in ``/dev/shm/<name>`` under a seqlock; any process reads them without
opening perf events (the reference's BPerf sharing role, BPerfEventsGroup.h).

    r = SharedCounters()           # default segment "dynolog_shared_counters"
    r.rebase(); work(); print(r.delta())   # {"instructions": ..., "cycles": ...}
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
