"""tools/pmc_traffic.py: the bench line's `roofline.traffic` source.  The
default bench line also launches k_mask / k_rv on the host phase's 4 Mi-word
batches, so only launches whose Grid_Size is the device-resident word count
may enter the per-launch figure (round 5: unfiltered, the average fell to
0.34 x algorithmic)."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
COLS = ["Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"]


def _csv(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        for grid, kernel, kib in rows:
            w.writerow({"Grid_Size": grid, "Kernel_Name": kernel, "Counter_Name": counter, "Counter_Value": kib})


def test_only_device_resident_launches_count(tmp_path):
    W, n = 1 << 20, 2
    algo = {"k_mask": (80 * n + 32) * W, "k_rv": (80 * n + 16) * W}
    big = "void amph::(anonymous namespace)::k_mask<2, true, true>(Fp, ...)"
    rv = "k_rv"
    # device-resident launches: FETCH (halved on gfx950) + WRITE = algorithmic
    fetch_rows = [(W, big, (algo["k_mask"] - 16 * W) / 2 / 1024)] * 3 + [(W, rv, (algo["k_rv"] - 16 * W) / 2 / 1024)] * 3
    write_rows = [(W, big, 16 * W / 1024)] * 3 + [(W, rv, 16 * W / 1024)] * 3
    # host-phase batch launches (a quarter of the words): must be ignored
    fetch_rows += [(W // 4, big, 1.0)] * 5 + [(W // 4, rv, 1.0)] * 5
    write_rows += [(W // 4, big, 1.0)] * 5 + [(W // 4, rv, 1.0)] * 5
    _csv(tmp_path / "f.csv", "FETCH_SIZE", fetch_rows)
    _csv(tmp_path / "w.csv", "WRITE_SIZE", write_rows)
    out = tmp_path / "traffic.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), "--words", str(W), "--parties", str(n), "--out", str(out)],
                   check=True, capture_output=True)
    got = json.loads(out.read_text())
    for k in ("k_mask", "k_rv"):
        e = got["%s_n%d_w%d" % (k, n, W)]
        assert e["hbm_bytes_per_launch"] == algo[k]
        assert e["ratio_to_algorithmic"] == 1.0


def test_launch_size_is_work_items_not_words(tmp_path):
    """rocprof's Grid_Size counts work-items: ceil(W / block) x block.  A word
    count that is no multiple of the block still selects its launches, an
    explicit --grid (a capped grid) selects others, and a run with no
    matching launch fails naming the sizes it saw."""
    W, n = 1_000_003, 2
    grid = -(-W // 256) * 256
    k = "k_mask"
    _csv(tmp_path / "f.csv", "FETCH_SIZE", [(grid, k, 10.0)] * 2 + [(4096, k, 99.0)])
    _csv(tmp_path / "w.csv", "WRITE_SIZE", [(grid, k, 5.0)] * 2 + [(4096, k, 99.0)])
    out = tmp_path / "t.json"
    cmd = [sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), str(tmp_path / "f.csv"), str(tmp_path / "w.csv"),
           "--words", str(W), "--parties", str(n), "--out", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    assert json.loads(out.read_text())["k_mask_n2_w%d" % W]["hbm_bytes_per_launch"] == (2 * 10.0 + 5.0) * 1024
    subprocess.run(cmd + ["--grid", "4096"], check=True, capture_output=True)
    assert json.loads(out.read_text())["k_mask_n2_w%d" % W]["hbm_bytes_per_launch"] == (2 * 99.0 + 99.0) * 1024
    r = subprocess.run(cmd[:-4] + ["--words", "77", "--parties", str(n), "--out", str(out)], capture_output=True,
                       text=True)
    assert r.returncode != 0 and "no FETCH_SIZE launch" in r.stderr and "4096" in r.stderr
