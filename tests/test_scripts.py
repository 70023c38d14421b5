"""Scripts and Python helpers (the reference has no tests for unitrace.py)."""
import importlib.util
import os
import subprocess
import sys

from dynolog_amd.utils import client

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load_unitrace():
    spec = importlib.util.spec_from_file_location("unitrace", os.path.join(REPO, "scripts/pytorch/unitrace.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_hostlist_expansion():
    ut = _load_unitrace()
    assert ut.expand_hostlist("gpu[01-03],login") == ["gpu01", "gpu02", "gpu03", "login"]
    assert ut.expand_hostlist("a[1,3-4]b") == ["a1b", "a3b", "a4b"]


def test_unitrace_dry_run_commands(native_built, tmp_path):
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts/pytorch/unitrace.py"),
                        "--hosts", "n[1-2]", "--job-id", "42", "-o", str(tmp_path), "--iterations", "5",
                        "--dry-run"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 2
    assert "--hostname n1" in lines[0] and "--job-id 42" in lines[0]
    assert "--iterations 5" in lines[0] and "--profile-start-iteration-roundup 1000" in lines[0]
    assert f"{tmp_path}/libkineto_trace_n2.json" in lines[1]


def test_client_config_matches_cli():
    cfg = client.kineto_config("/tmp/t.json", duration_ms=500)
    assert cfg == "PROFILE_START_TIME=0\nACTIVITIES_LOG_FILE=/tmp/t.json\nACTIVITIES_DURATION_MSECS=500"
    cfg = client.kineto_config("/tmp/t.json", iterations=3, start_iteration_roundup=10)
    assert cfg.endswith("PROFILE_START_ITERATION_ROUNDUP=10\nACTIVITIES_ITERATIONS=3")
    assert client.trace_files("/x/t.json", [5, 6]) == ["/x/t_5.json", "/x/t_6.json"]


def test_linear_model_example_runs_on_cpu():
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "pytorch", "linear_model_example.py"),
                        "--iterations", "3", "--batch", "8", "--dim", "16", "--device", "cpu",
                        "--print-every", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("PID ")
    assert "iter 3 loss" in r.stdout
