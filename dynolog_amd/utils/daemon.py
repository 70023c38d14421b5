"""Launch / stop a `dynolog` daemon subprocess (tests, benchmarks, SLURM
wrapper).  The daemon is the in-tree C++ binary (build/dynolog)."""
from __future__ import annotations

import os
import re
import signal
import subprocess
import tempfile
import time
from typing import Optional, Sequence

from dynolog_amd import _native
from dynolog_amd.utils import client


class DaemonProcess:
    """Context manager: starts `dynolog --port 0 ...`, discovers the RPC port
    from its log, stops it with SIGTERM (clean shutdown path)."""

    def __init__(self, args: Sequence[str] = (), env: Optional[dict] = None,
                 log_path: Optional[str] = None, start_timeout: float = 20.0):
        _native.ensure_built(gpu=False)
        self.args = list(args)
        self.env = dict(os.environ, **(env or {}))
        self.log_path = log_path or tempfile.mktemp(prefix="dynolog_", suffix=".log")
        self.start_timeout = start_timeout
        self.proc: Optional[subprocess.Popen] = None
        self.port: Optional[int] = None

    def start(self) -> "DaemonProcess":
        cmd = [_native.binary("dynolog"), "--port", "0", *self.args]
        self._log = open(self.log_path, "w")
        self.proc = subprocess.Popen(cmd, stdout=self._log, stderr=subprocess.STDOUT, env=self.env)
        deadline = time.time() + self.start_timeout
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"dynolog exited rc={self.proc.returncode}:\n{self.log()}")
            m = re.search(r"Listening to connections on port (\d+)", self.log())
            if m:
                self.port = int(m.group(1))
                return self
            time.sleep(0.05)
        self.stop()
        raise RuntimeError("dynolog did not start:\n" + self.log())

    def log(self) -> str:
        try:
            with open(self.log_path) as f:
                return f.read()
        except OSError:
            return ""

    def rpc(self, req, timeout: float = 10.0) -> Optional[dict]:
        return client.call(req, port=self.port, timeout=timeout)

    def stop(self, timeout: float = 10.0) -> int:
        if self.proc is None:
            return 0
        if self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        self._log.close()
        return self.proc.returncode

    def __enter__(self) -> "DaemonProcess":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()
