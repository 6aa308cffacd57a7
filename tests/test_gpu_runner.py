"""tools/gpu_run.sh, the one GPU-box runner: steps separated by `::`, each
under its own time limit, output under gpurun_out/$TAG/<n>_<kind>.*, and the
first failing step ends the call (nothing more runs after a fault or a
timeout).  Exercised here with CPU-only `py` steps in a scratch root."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "tools", "gpu_run.sh")


def _run(tmp_path, *steps):
    env = dict(os.environ, GRAFT_REPO_ROOT=str(tmp_path), TAG="t")
    r = subprocess.run(["bash", RUNNER] + list(steps), env=env, capture_output=True, text=True, timeout=120)
    status = (tmp_path / "gpurun_out" / "t" / "status.txt").read_text().splitlines()
    return r.returncode, status


def test_steps_run_in_order_each_logged(tmp_path):
    rc, status = _run(tmp_path, "py", "30", "-c", "print('one')", "::", "py", "30", "-c", "print('two')")
    assert rc == 0
    assert [ln.split()[:2] for ln in status[1:3]] == [["1", "py"], ["2", "py"]] and status[-1].startswith("end rc=0")
    assert "one" in (tmp_path / "gpurun_out" / "t" / "1_py.log").read_text()
    assert "two" in (tmp_path / "gpurun_out" / "t" / "2_py.log").read_text()


def test_first_failure_ends_the_call(tmp_path):
    rc, status = _run(tmp_path, "py", "30", "-c", "import sys; sys.exit(3)", "::", "py", "30", "-c", "print('never')")
    assert rc == 3
    assert status[1].split()[:2] == ["1", "py"] and status[1].endswith(status[1].split()[-1])
    assert "rc=3" in status[1] and not (tmp_path / "gpurun_out" / "t" / "2_py.log").exists()


def test_a_step_over_its_limit_is_killed_and_ends_the_call(tmp_path):
    rc, status = _run(tmp_path, "py", "2", "-c", "import time; time.sleep(30)", "::", "py", "30", "-c", "print(1)")
    assert rc == 124 and "rc=124" in status[1]
    assert not (tmp_path / "gpurun_out" / "t" / "2_py.log").exists()


def test_unknown_step_kind_fails(tmp_path):
    rc, status = _run(tmp_path, "frobnicate")
    assert rc != 0 and "unknown step kind" in (tmp_path / "gpurun_out" / "t" / "1_frobnicate.log").read_text()
