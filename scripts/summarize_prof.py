#!/usr/bin/env python3
"""Summarise a scripts/gpu_prof.sh output directory into profiles/<name>/SUMMARY.md plus the
raw rocprofv3 CSVs worth keeping (kernel stats, per-dispatch PMC rows of hgd kernels).

    python scripts/summarize_prof.py gpurun_out/prof3 profiles/r01_synthetic_d64
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    lines = [f"# rocprofv3 summary: {os.path.basename(dst)}", ""]
    bench = os.path.join(src, "bench.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(dst, "bench.json"))
        b = json.loads(open(bench).read().strip().splitlines()[-1])
        lines += ["## bench.py line (same box, same workload)", "",
                  f"- value: **{b['value']} {b['unit']}**, {b['ms_per_step']} ms/step, "
                  f"workload `{b['config']['workload']}`",
                  f"- roofline: achieved {b['roofline']['achieved']} GB/s of "
                  f"{b['roofline']['peak']} ({100 * b['roofline']['frac']:.1f} %), "
                  f"avg hgd_spmm launch {b['roofline']['avg_launch_ms']} ms, "
                  f"algorithmic {b['roofline']['algorithmic_bytes_per_launch'] / 1e9:.2f} GB/launch",
                  f"- PMC traffic: {b['roofline'].get('traffic')} B/launch "
                  f"({b['roofline'].get('traffic_note', '')})", ""]
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        rows = list(csv.DictReader(open(stats[0])))
        lines += ["## Kernel stats (`rocprofv3 --kernel-trace --stats`)", "",
                  "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
        for r in rows[:10]:
            lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | "
                         f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} |")
        spmm = [r for r in rows if "spmm_kernel" in r["Name"]]
        if spmm:
            calls = sum(int(r["Calls"]) for r in spmm)
            tot = sum(float(r["TotalDurationNs"]) for r in spmm)
            lines += ["", f"All `hgd::spmm_kernel` instantiations: {calls} calls, "
                      f"average {tot / calls / 1e6:.4f} ms per launch (compare bench "
                      f"`roofline.avg_launch_ms`).", ""]
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(src, f"pmc_{ctr}", "*counter_collection.csv"))
        if not f:
            continue
        vals = {}
        keep = []
        for r in csv.DictReader(open(f[0])):
            if "hgd::" in r["Kernel_Name"]:
                keep.append(r)
                vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
        with open(os.path.join(dst, f"pmc_{ctr}.csv"), "w", newline="") as fh:
            if keep:
                w = csv.DictWriter(fh, fieldnames=list(keep[0].keys()))
                w.writeheader()
                w.writerows(keep)
        lines += [f"## {ctr} per dispatch (KB, raw counter; gfx950 FETCH_SIZE reads ½ of wide "
                  f"streaming reads, so HBM read bytes ≈ 2 × FETCH_SIZE × 1024)", "",
                  "| kernel | dispatches | mean KB |", "|---|---|---|"]
        for k, v in vals.items():
            lines.append(f"| `{k[:70]}` | {len(v)} | {statistics.mean(v):.0f} |")
        lines.append("")
    open(os.path.join(dst, "SUMMARY.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
