"""Host CPU PMU co-sampling next to the GPU counters (BASELINE config 5).

Runs the in-tree `dynolog --enable_perf_monitor` (src/pmu: perf_event on the
AMD EPYC core / L3 / UMC PMUs) for the duration of a training job and lets
the caller pause it together with the GPU agent, so the interleaved A/B
windows of bench.py price both samplers at once.

Targets, tried in order:
  1. system-wide (every CPU; the only mode that can open the uncore
     `l3_cache` / `dram_bandwidth` metrics) -- needs perf_event_paranoid <= 0
     or CAP_PERFMON, like the reference's PerfMonitor (dynolog/src/
     PerfMonitor.cpp:24-63, which only opens system-wide groups);
  2. per process (`--perf_monitor_pids` = the training ranks on this node),
     core metrics only -- works under paranoid 1-2 for the daemon user's own
     processes;
  3. unavailable: the summary carries the kernel's reason (paranoid 3, as on
     hosts that forbid unprivileged perf_event_open entirely).

Metrics are kernel-multiplexed in one group (`--perf_monitor_mux=false`), so
every record carries every metric plus `<id>_mux_ratio` (time running /
time enabled) whenever the core PMU had to time-share its counters.
"""
from __future__ import annotations

import collections
import math
import time
from typing import Optional, Sequence

DEFAULT_METRICS = ("instructions,cycles,l2_cache_misses,tlb_misses,l3_cache,dram_bandwidth")


class HostPmuCosampler:
    def __init__(self, metrics: str = DEFAULT_METRICS, interval_s: int = 1,
                 extra_args: Sequence[str] = (), start_timeout_s: float = 30.0):
        self.metrics = metrics
        self.extra_args = list(extra_args)
        self.start_timeout_s = start_timeout_s
        self.interval_s = max(1, int(interval_s))
        self.daemon = None
        self.mode: Optional[str] = None
        self.reason = ""
        self.active: list = []

    def _start(self, extra: Sequence[str]):
        from dynolog_amd.utils.daemon import DaemonProcess
        d = DaemonProcess(["--enable_perf_monitor", "--perf_monitor_mux=false",
                           "--perf_monitor_reporting_interval_s", str(self.interval_s),
                           "--perf_monitor_metrics", self.metrics, *self.extra_args, *extra])
        d.start()
        # "starting": the daemon serves RPCs before its counters are open
        # (opening system-wide groups on every CPU takes a while); poll.
        deadline = time.monotonic() + self.start_timeout_s
        while True:
            st = d.rpc({"fn": "setPerfMonitor"}) or {}
            if st.get("status") != "starting" or time.monotonic() > deadline:
                break
            time.sleep(0.05)
        if st.get("status") == "ok":
            return d, st
        d.stop()
        return None, st

    def start(self, pids: Sequence[int] = ()) -> "HostPmuCosampler":
        """Never raises: on any failure the sampler is left off with a reason."""
        try:
            d, st = self._start([])
            self.mode = "system-wide"
            if d is None and pids:
                first = st.get("status", "")
                d, st = self._start(["--perf_monitor_pids", ",".join(str(p) for p in pids)])
                self.mode = "per-process"
                if d is None:
                    st = {"status": f"{first}; per-process: {st.get('status', '')}"}
            if d is None:
                self.mode = None
                self.reason = str(st.get("status", "unavailable"))
                return self
            self.daemon, self.active = d, list(st.get("active", []))
        except Exception as e:  # noqa: BLE001 - co-sampling must never break the job
            self.mode, self.reason = None, f"failed: {e}"
        return self

    @property
    def running(self) -> bool:
        return self.daemon is not None

    def set_enabled(self, on: bool) -> None:
        if self.daemon is not None:
            try:
                self.daemon.rpc({"fn": "setPerfMonitor", "enable": bool(on)}, timeout=5.0)
            except Exception:  # noqa: BLE001
                pass

    def records(self) -> list:
        if self.daemon is None:
            return []
        r = self.daemon.rpc({"fn": "getMetrics", "collector": "perf", "last": 100000}) or {}
        return list(r.get("records", []))

    def summary(self) -> dict:
        """Never raises (the caller prints its result line right after)."""
        if self.daemon is None:
            return {"status": "unavailable", "reason": self.reason}
        try:
            recs = self.records()
        except Exception as e:  # noqa: BLE001 - e.g. the daemon died mid-run
            return {"status": "failed", "mode": self.mode, "reason": f"records: {e}"}
        sums, counts = collections.defaultdict(float), collections.Counter()
        for r in recs:
            for k, v in r.items():
                if k in ("pid", "ts_ms") or not isinstance(v, (int, float)) or not math.isfinite(v):
                    continue
                sums[k] += float(v)
                counts[k] += 1
        means = {k: round(sums[k] / counts[k], 4) for k in sorted(sums)}
        return {
            "status": "ok", "mode": self.mode, "interval_s": self.interval_s,
            "active_metrics": self.active, "records": len(recs),
            "pids": sorted({r["pid"] for r in recs if "pid" in r}),
            "mean": {k: v for k, v in means.items() if not k.endswith("_mux_ratio")},
            "mux_ratio": {k[: -len("_mux_ratio")]: v for k, v in means.items()
                          if k.endswith("_mux_ratio")},
        }

    def stop(self) -> None:
        if self.daemon is not None:
            try:
                self.daemon.stop()
            finally:
                self.daemon = None
