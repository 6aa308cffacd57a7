"""bench.py's host-memory probe (memory_limits): the binding limit is the
smallest headroom along this process's cgroup chain -- its own cgroup and
every ancestor, v2 or v1 -- not only the hierarchy's root (a lease's limit
may sit on an intermediate level).  Fake cgroup trees under tmp_path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

G = 1 << 30


def _w(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        fh.write(text)


def test_v2_limit_on_an_ancestor_binds(tmp_path, monkeypatch):
    r = tmp_path / "cg"
    _w(str(r / "cgroup.controllers"), "memory\n")
    _w(str(r / "memory.max"), "max\n")
    _w(str(r / "lease" / "memory.max"), "%d\n" % (100 * G))
    _w(str(r / "lease" / "memory.current"), "%d\n" % (30 * G))
    _w(str(r / "lease" / "memory.stat"), "anon 1\ninactive_file %d\n" % (10 * G))
    _w(str(r / "lease" / "job" / "memory.max"), "max\n")
    _w(str(r / "lease" / "job" / "memory.current"), "%d\n" % G)
    _w(str(tmp_path / "self_cgroup"), "0::/lease/job\n")
    monkeypatch.setenv("AMPH_BENCH_CGROUP_ROOT", str(r))
    monkeypatch.setenv("AMPH_BENCH_PROC_CGROUP", str(tmp_path / "self_cgroup"))
    monkeypatch.setenv("AMPH_BENCH_MEM_AVAILABLE_BYTES", str(1000 * G))
    lim = bench.memory_limits()
    assert lim["mem_limit_bytes"] == 100 * G and lim["mem_limit_used_bytes"] == 20 * G
    assert lim["headroom_bytes"] == 80 * G and lim["source"]["limit"].endswith("lease")


def test_v2_tighter_own_limit_wins(tmp_path, monkeypatch):
    r = tmp_path / "cg"
    _w(str(r / "cgroup.controllers"), "memory\n")
    _w(str(r / "lease" / "memory.max"), "%d\n" % (100 * G))
    _w(str(r / "lease" / "memory.current"), "%d\n" % (10 * G))
    _w(str(r / "lease" / "job" / "memory.max"), "%d\n" % (20 * G))
    _w(str(r / "lease" / "job" / "memory.current"), "%d\n" % (5 * G))
    _w(str(tmp_path / "self_cgroup"), "0::/lease/job\n")
    monkeypatch.setenv("AMPH_BENCH_CGROUP_ROOT", str(r))
    monkeypatch.setenv("AMPH_BENCH_PROC_CGROUP", str(tmp_path / "self_cgroup"))
    lim = bench.memory_limits()
    assert lim["mem_limit_bytes"] == 20 * G and lim["headroom_bytes"] <= 15 * G


def test_v1_memory_controller_path(tmp_path, monkeypatch):
    r = tmp_path / "cg"
    _w(str(r / "memory" / "memory.limit_in_bytes"), "9223372036854771712\n")  # root: unlimited
    _w(str(r / "memory" / "pod" / "memory.limit_in_bytes"), "%d\n" % (64 * G))
    _w(str(r / "memory" / "pod" / "memory.usage_in_bytes"), "%d\n" % (4 * G))
    _w(str(r / "memory" / "pod" / "memory.stat"), "total_inactive_file %d\n" % G)
    _w(str(tmp_path / "self_cgroup"), "4:memory:/pod\n1:cpu:/\n0::/\n")
    monkeypatch.setenv("AMPH_BENCH_CGROUP_ROOT", str(r))
    monkeypatch.setenv("AMPH_BENCH_PROC_CGROUP", str(tmp_path / "self_cgroup"))
    monkeypatch.setenv("AMPH_BENCH_MEM_AVAILABLE_BYTES", str(1000 * G))
    lim = bench.memory_limits()
    assert lim["mem_limit_bytes"] == 64 * G and lim["headroom_bytes"] == 61 * G


def test_no_limit_anywhere_leaves_mem_available(tmp_path, monkeypatch):
    r = tmp_path / "cg"
    _w(str(r / "cgroup.controllers"), "memory\n")
    _w(str(r / "memory.max"), "max\n")
    _w(str(tmp_path / "self_cgroup"), "0::/\n")
    monkeypatch.setenv("AMPH_BENCH_CGROUP_ROOT", str(r))
    monkeypatch.setenv("AMPH_BENCH_PROC_CGROUP", str(tmp_path / "self_cgroup"))
    monkeypatch.setenv("AMPH_BENCH_MEM_AVAILABLE_BYTES", str(7 * G))
    lim = bench.memory_limits()
    assert lim["mem_limit_bytes"] is None and lim["headroom_bytes"] == 7 * G
