"""bench.py's per-rank phase deadlines (dynolog_amd/utils/watchdog.py): a
rank that hangs must end the run inside the deadline, non-zero, with the
hung rank named -- rehearsed on CPU (gloo, 4 ranks, the tiny model)."""
import io
import os
import subprocess
import sys
import time

from dynolog_amd.utils.watchdog import EXIT_CODE, PhaseWatchdog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_phase_deadline_fires_with_progress(tmp_path):
    out = io.StringIO()
    code = []
    wd = PhaseWatchdog(rank=1, world=3, total_s=0, poll_s=0.02, hb_dir=str(tmp_path), stream=out,
                       exit_fn=code.append)
    # two peers' heartbeats: rank 0 one stage further on, rank 2 at the same point
    (tmp_path / "rank0.json").write_text('{"rank": 0, "phase": "w", "step": 4, "stage": "backward"}')
    (tmp_path / "rank2.json").write_text('{"rank": 2, "phase": "w", "step": 4, "stage": "backward"}')
    wd.progress(4, "start")
    wd.phase("timed window 1 (5 steps)", 0.1)
    deadline = time.time() + 5
    while not code and time.time() < deadline:
        time.sleep(0.02)
    assert code == [EXIT_CODE]
    text = out.getvalue()
    assert "phase 'timed window 1 (5 steps)' exceeded its 0 s deadline" in text or "exceeded its" in text, text
    assert "this rank was at step 4 (start)" in text, text
    assert "suspect rank 1 (least progress: step 4, start)" in text, text


def test_no_suspect_when_all_ranks_agree(tmp_path):
    out = io.StringIO()
    code = []
    wd = PhaseWatchdog(rank=0, world=2, total_s=0.1, poll_s=0.02, hb_dir=str(tmp_path), stream=out,
                       exit_fn=code.append)
    (tmp_path / "rank1.json").write_text('{"rank": 1, "phase": "p", "step": 2, "stage": "forward"}')
    wd.progress(2, "forward")
    deadline = time.time() + 5
    while not code and time.time() < deadline:
        time.sleep(0.02)
    assert code == [EXIT_CODE]
    assert "overall" in out.getvalue() and "suspect" not in out.getvalue(), out.getvalue()


def test_phase_cleared_deadline_does_not_fire(tmp_path):
    code = []
    wd = PhaseWatchdog(rank=0, world=1, total_s=0, poll_s=0.02, hb_dir=str(tmp_path), stream=io.StringIO(),
                       exit_fn=code.append)
    wd.phase("fast", 0.3)
    wd.phase("next", 30.0)  # the first phase ended in time
    time.sleep(0.5)
    wd.stop()
    assert code == []
    assert not (tmp_path / "rank0.json").exists()  # heartbeat removed at stop


def test_four_rank_hang_ends_within_deadline_naming_the_rank():
    """bench.py --gpus 4 on CPU (gloo) with rank 2 hanging in its own work at
    step 3: every rank's window deadline fires, the job exits non-zero well
    inside the overall deadline, and the output names rank 2."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--model", "tiny",
           "--micro-batch", "2", "--seq-len", "64", "--gpus", "4", "--steps", "5", "--warmup", "1",
           "--skip-baseline", "--fault-hang", "2@3", "--step-timeout-s", "2", "--phase-base-s", "8",
           "--deadline-s", "90"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd="/tmp")
    took = time.time() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    assert took < 90, took
    err = r.stderr
    # whichever rank's deadline fires first (torchrun then ends the others)
    # reports the phase, every rank's progress and the suspect
    assert "phase 'timed window 1 (5 steps)' exceeded its 18 s deadline" in err, err[-4000:]
    assert "rank 2: phase timed window 1 (5 steps), step 3 (start)" in err, err[-4000:]
    assert "suspect rank 2 (least progress: step 3, start)" in err, err[-4000:]
