"""bench.py on the GPU, as the driver runs it (the N > 1 shape rehearsed on
one GPU): two self-spawned ranks under torch.distributed.run with gloo, both
driving cuda:0, run the C4 workload strong-scaled (two 2^25-word shards), the
host_memory phase (a 1 Mi-word share per rank here) and the root-held
scatter/gather phase.  The HIP kernels run under a real process group and
every check the line carries must hold: per-step verdicts all-reduced to the
global index, outputs checked against the generated secrets and a Python
recomputation, the gathered masked words equal to one K_MASK launch over the
root's whole arrays."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_line_under_a_process_group():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    argv = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--same-device",
            "--steps", "5", "--warmup", "2", "--sg-steps", "1", "--sg-warmup", "0", "--host-words",
            str(1 << 20), "--host-steps", "2", "--no-cpu-baseline"]
    r = subprocess.run(argv, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["verified"] is True, line["verify_checks"]
    assert line["n_gpus"] == 2 and line["config"]["words_total"] == 1 << 26
    assert all(line["verify_checks"].values()) and line["verify_checks"]["all_ranks"]
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    assert line["ranks_summary"]["pg_world_size"] == 2
    hm = line["host_memory"]
    assert hm["verified"] is True and hm["words_per_rank"] == 1 << 20
    assert hm["words_per_s"] > 0 and hm["frac_of_link"] > 0
    sg = line["scatter_gather"]
    assert sg["verified"] is True and all(sg["verify_checks"].values()), sg
