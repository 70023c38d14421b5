"""Child workload processes for the daemon / agent integration tests.

A test that asks the daemon to capture a child (a kernel trace, SQTT, RCCL
calls, counter records) must only start once the child's workload is WARM:
its first GEMM done (hipBLASLt code objects loaded, the first launch's
seconds of one-time cost paid) and, for agent children, the agent sampling.
So every child script prints its ready line ("PID <pid>") only after that,
and the parent waits for it with a deadline, with the child's stdout and
stderr in any failure message.  Output goes to files, never to pipes: a
chatty child (RCCL banners, agent log lines) can then never block on a full
pipe while the parent is busy elsewhere.

Pattern: the reference's fork-based client/server handshake, where the
parent acts only after the child reported it is set up
(/root/reference/dynolog/tests/tracing/IPCMonitorTest.cpp:60-75).
"""
import os
import subprocess
import sys
import tempfile
import textwrap
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Warm-up snippets for child scripts (indented to the script's top level).
# A bf16 GEMM and a sync: the first hipBLASLt call loads its code objects.
WARM_GEMM = "_w = torch.randn(1024, 1024, device='cuda', dtype=torch.bfloat16); _w = _w @ _w; torch.cuda.synchronize()"
# An agent `a` has taken samples (its sampler thread and counting context are up).
WARM_AGENT = ("_t = time.time()\n"
              "while a.stats()['samples_taken'] == 0 and time.time() - _t < 30: time.sleep(0.01)")


class Child:
    """A child Python process whose ready line ("PID <pid>") marks a warm workload."""

    def __init__(self, code, args=(), env=None, ready="PID"):
        self.ready = ready
        self._dir = tempfile.mkdtemp(prefix="dychild")
        self.out_path = os.path.join(self._dir, "stdout")
        self.err_path = os.path.join(self._dir, "stderr")
        e = dict(os.environ if env is None else env)
        e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
        e.setdefault("PYTHONUNBUFFERED", "1")
        self._out = open(self.out_path, "w")
        self._err = open(self.err_path, "w")
        self.p = subprocess.Popen([sys.executable, "-c", textwrap.dedent(code), *map(str, args)],
                                  env=e, stdout=self._out, stderr=self._err, text=True)
        self.pid = None

    def stdout(self) -> str:
        with open(self.out_path) as f:
            return f.read()

    def stderr(self) -> str:
        with open(self.err_path) as f:
            return f.read()

    def tails(self, n=3000) -> str:
        rc = self.p.poll()
        return (f"[child pid {self.p.pid} rc={rc}]\n--- stdout ---\n{self.stdout()[-n:]}\n"
                f"--- stderr ---\n{self.stderr()[-n:]}")

    def wait_ready(self, timeout=180.0) -> int:
        """The child's pid once it printed its ready line; AssertionError (with
        the child's output) if it exits or the deadline passes first."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            for line in self.stdout().splitlines():
                if line.startswith(self.ready + " "):
                    self.pid = int(line.split()[1])
                    return self.pid
            if self.p.poll() is not None:
                raise AssertionError("child exited before it was ready\n" + self.tails())
            time.sleep(0.05)
        raise AssertionError(f"child not ready within {timeout:.0f} s\n" + self.tails())

    def lines(self, prefix) -> list:
        return [l for l in self.stdout().splitlines() if l.startswith(prefix)]

    def finish(self, done_flag=None, timeout=60.0) -> int:
        """Ask the child to end (touch its DONE_FLAG), wait bounded, kill if it
        hangs (AssertionError naming it).  Returns the exit code."""
        if done_flag:
            open(done_flag, "w").close()
        try:
            rc = self.p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            self.kill()
            raise AssertionError(f"child hung at exit (> {timeout:.0f} s)\n" + self.tails(6000))
        self._close()
        return rc

    def kill(self):
        if self.p.poll() is None:
            self.p.kill()
            try:
                self.p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                pass
        self._close()

    def _close(self):
        for f in (self._out, self._err):
            try:
                f.close()
            except OSError:
                pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.kill()
        return False
