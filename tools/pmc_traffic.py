"""Per-launch HBM traffic from rocprofv3 PMC passes -> profiles/traffic.json.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV --words W --parties N [--out profiles/traffic.json]

FETCH_SIZE and WRITE_SIZE come from separate passes (they cannot share one on
gfx950).  Per MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE reports exactly
half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Units: KiB.
"""
import argparse
import collections
import csv
import json
import os


def kernel_short(name):
    """'void amph::(anonymous namespace)::k_rv<2, true, true>(...)' or a
    truncated 'k_rv' -> 'k_rv'."""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("<")[0].split("::")[-1].strip()


BLOCKS = (64, 128, 256, 512, 1024)


def launch_sizes(words, grid=None):
    """Grid_Size values (work-items) a W-word launch can have: rocprof counts
    work-items, ceil(W / block) x block for the library's block sizes, or
    exactly `grid` when given (a grid cap, AMPH_GRID_CAP, makes it smaller)."""
    if grid is not None:
        return {grid}
    return {-(-words // b) * b for b in BLOCKS}


def per_kernel(path, counter, words=None, grid=None):
    """Average per launch over the launches of a W-word call (the default
    bench line also launches k_mask / k_rv on the host phase's 4 Mi-word
    batches, which must not enter the device-resident figure).  Fails,
    naming the sizes it saw, when no launch matches."""
    vals = collections.defaultdict(list)
    seen = collections.Counter()
    sizes = launch_sizes(words, grid) if words is not None else None
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        g = int(r.get("Grid_Size") or -1)
        k = kernel_short(r["Kernel_Name"])
        seen[(k, g)] += 1
        if sizes is not None and g not in sizes:
            continue
        vals[k].append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit("%s: no %s launch with Grid_Size in %s; launches seen (kernel, Grid_Size): %s -- "
                         "pass --grid" % (path, counter, sorted(sizes or []), dict(seen.most_common(8))))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--words", type=int, required=True)
    ap.add_argument("--parties", type=int, required=True)
    ap.add_argument("--grid", type=int, default=None,
                    help="the launches' Grid_Size (work-items) when not ceil(W / block) x block")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json"))
    a = ap.parse_args()
    f = per_kernel(a.fetch_csv, "FETCH_SIZE", a.words, a.grid)
    w = per_kernel(a.write_csv, "WRITE_SIZE", a.words, a.grid)
    algo = {"k_rv": 80 * a.parties + 16, "k_mask": 80 * a.parties + 32}
    out = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for k in ("k_mask", "k_rv"):
        if k not in f or k not in w:
            continue
        fetch = 2 * f[k] * 1024
        write = w[k] * 1024
        out["%s_n%d_w%d" % (k, a.parties, a.words)] = {
            "hbm_bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch,
            "write_bytes": write, "algorithmic_bytes": algo[k] * a.words,
            "ratio_to_algorithmic": (fetch + write) / (algo[k] * a.words),
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH x2 (gfx950)"}
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
