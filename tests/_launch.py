"""Helpers to run multi-rank workers from a single pytest process."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN = os.path.join(REPO, "scripts", "mpirun")


def run_ranks(n, argv, timeout=240, env=None, check=True):
    """Run ``argv`` on ``n`` ranks via the framework launcher; returns CompletedProcess."""
    e = dict(os.environ)
    e.setdefault("CCMPI_TIMEOUT", str(max(30, timeout - 10)))
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    if env:
        e.update(env)
    cmd = [MPIRUN, "-n", str(n), "--timeout", str(timeout - 5)] + list(argv)
    r = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=timeout + 30)
    if check and r.returncode != 0:
        raise AssertionError(f"{n}-rank run failed (rc={r.returncode}):\nSTDOUT:\n{r.stdout[-6000:]}\n"
                             f"STDERR:\n{r.stderr[-6000:]}")
    return r


def py(*args):
    return [sys.executable, *args]
