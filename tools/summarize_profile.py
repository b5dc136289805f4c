#!/usr/bin/env python3
"""Turns a tools/profile.sh output directory into committed evidence:
  profiles/<round>/<tag>_kernel_stats.csv   rocprofv3 --stats summary (per-kernel average duration)
  profiles/<round>/<tag>_summary.md         fill-kernel duration, PMC bytes per launch, roofline
  profiles/traffic.json                     {workload: HBM bytes per fill launch} read by bench.py

Per-launch HBM traffic = (2 x FETCH_SIZE + WRITE_SIZE) of the fill kernel, averaged over its
dispatches. rocprofv3 reports both in KiB. Corrections per MI355X_MICROARCH.md §HBM:
  * FETCH_SIZE counts half the bytes of 16-B-per-lane loads on gfx950; the fill kernel's reads are
    its text-code global_load_dwordx4 (16 B/lane), so FETCH_SIZE is doubled;
  * WRITE_SIZE is checked against the known byte count of the direction planes (the plan's mask
    bytes, reported by bench.py as direction_bytes_physical_per_launch).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter_per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for fpath in files:
        for r in rows(fpath):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            per.setdefault(name, {}).setdefault(r["Dispatch_Id"], 0.0)
            per[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in per.items()}


def main():
    src, rnd, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    st = rows(stats)
    fill = next(r for r in st if "fill_kernel" in r["Name"] or "fill_pair_kernel" in r["Name"])
    avg_ns = float(fill["AverageNs"])
    bench = json.loads(open(os.path.join(src, "bench_trace.json")).read().strip().splitlines()[-1])
    wl = bench["config"]["workload"]
    cells = bench["config"]["text_len"] * bench["config"]["pattern_len"] * bench["config"].get("pairs_per_gpu", 1)
    if "pairs_total" in bench["config"]:
        cells = bench["config"]["text_len"] * bench["config"]["pattern_len"] * bench["config"]["pairs_total"] // bench["n_gpus"]
    w = counter_per_kernel(os.path.join(src, "pmc_write"), "WRITE_SIZE")
    f = counter_per_kernel(os.path.join(src, "pmc_fetch"), "FETCH_SIZE")
    kname = next(k for k in w if "fill_kernel" in k or "fill_pair_kernel" in k)
    wb = w[kname] * 1024.0
    fb = f.get(kname, 0.0) * 1024.0 * 2.0  # gfx950: FETCH_SIZE = half the bytes of 16-B/lane loads
    traffic = wb + fb
    planes = float(bench.get("direction_bytes_physical_per_launch") or 0)
    achieved = cells / (avg_ns * 1e-9) / 1e9
    lines = [
        f"# {tag}: {wl}",
        "",
        f"- fill kernel `{fill['Name']}`: {fill['Calls']} calls, average {avg_ns / 1e6:.4f} ms "
        f"(min {float(fill['MinNs']) / 1e6:.4f}, max {float(fill['MaxNs']) / 1e6:.4f})",
        f"- cells per launch: {cells:,} -> {cells / avg_ns:.1f} GCUPS; algorithmic bytes (1 B/cell) "
        f"{achieved:.1f} GB/s = {achieved / 8000:.4f} of 8 TB/s",
        f"- PMC per launch: WRITE_SIZE {wb / 1e6:.2f} MB, FETCH_SIZE x2 {fb / 1e6:.2f} MB, total {traffic / 1e6:.2f} MB "
        f"({traffic / cells:.4f} B/cell physical vs 1 B/cell algorithmic)",
        f"- WRITE_SIZE calibration: direction planes of one launch are {planes / 1e6:.2f} MB "
        f"(2 bits/cell incl. padding steps); WRITE_SIZE / planes = {wb / planes if planes else float('nan'):.4f}",
        f"- bench line (trace run): {json.dumps({k: bench[k] for k in ('value', 'ms_per_step')})}",
        "",
        "All kernels (rocprofv3 --stats):",
        "",
        "| kernel | calls | avg ms | share |",
        "|---|---|---|---|",
    ]
    for r in st:
        lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.1f}% |")
    open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    t = json.load(open(tpath)) if os.path.exists(tpath) else {}
    t[wl] = {"bytes_per_launch": round(traffic), "write_bytes": round(wb), "fetch_bytes": round(fb),
             "source": f"profiles/{rnd}/{tag}_summary.md (rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE, separate passes)"}
    json.dump(t, open(tpath, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
