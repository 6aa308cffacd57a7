"""Summarise rocprofv3 --pmc CSVs per kernel: the average per dispatch of
every counter, and the ratios that say what bounds a kernel.

    python tools/pmc_summary.py DIR_OR_CSV [...] [--kernels k_mask_b64,k_rv_b64] [--words W]

Ratios (counter semantics per MI355X_MICROARCH.md §rocprofv3 PMC slots):
  wait / wave cycles           SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barrier)
  VALU-active / wave cycles    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both in quad-cycles)
  LDS bank-conflict share      SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  VALU instructions per word   SQ_INSTS_VALU x 64 / words (lane-instructions per word)
FETCH_SIZE is doubled (gfx950 counts a wide streaming read at half its bytes)
and WRITE_SIZE taken as is; both are KiB."""
import argparse
import collections
import csv
import glob
import json
import os


def rows(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                          recursive=True)
    for f in files:
        yield from csv.DictReader(open(f))


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("<")[0].split("::")[-1].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--kernels", default="")
    ap.add_argument("--words", type=int, default=0)
    a = ap.parse_args()
    want = set(k for k in a.kernels.split(",") if k)
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for p in a.paths:
        for r in rows(p):
            k = short(r["Kernel_Name"])
            if want and k not in want:
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"VGPR": r.get("VGPR_Count"), "LDS": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size"),
                       "wg": r.get("Workgroup_Size")}
    out = {}
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), **meta[k],
             "per_dispatch": {c: float("%.4g" % x) for c, x in sorted(avg.items())}}
        g = avg.get
        if g("SQ_WAVE_CYCLES"):
            if g("SQ_WAIT_ANY") is not None:
                d["wait_over_wave_cycles"] = round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 3)
            if g("SQ_ACTIVE_INST_VALU") is not None:
                d["valu_active_over_wave_cycles"] = round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 3)
            if g("SQ_WAIT_INST_ANY") is not None:
                d["issue_stall_over_wave_cycles"] = round(g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), 3)
        if g("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_share"] = round(g("SQ_LDS_BANK_CONFLICT", 0) / g("SQ_LDS_IDX_ACTIVE"), 3)
        if a.words and g("SQ_INSTS_VALU"):
            d["valu_lane_instructions_per_word"] = round(64 * g("SQ_INSTS_VALU") / a.words, 1)
        if g("FETCH_SIZE") is not None:
            d["fetch_bytes_corrected"] = 2 * g("FETCH_SIZE") * 1024
        if g("WRITE_SIZE") is not None:
            d["write_bytes"] = g("WRITE_SIZE") * 1024
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
