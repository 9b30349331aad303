#!/usr/bin/env python3
"""Summarise rocprofv3's SQLite output (run_results.db): per kernel the dispatch count, mean /
min duration and grid, and — for a --pmc pass — the mean of every collected counter per
dispatch. Usage: rocpd_summary.py DB [DB ...] [--match SUBSTR]."""
import argparse
import collections
import sqlite3


def summarize(path, match=None):
    c = sqlite3.connect(path)
    sym = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select id, kernel_id, start, end, grid_size_x, workgroup_size_x "
                     "from rocpd_kernel_dispatch").fetchall()
    pmc_names = {r[0]: r[1] for r in c.execute("select id, name from rocpd_info_pmc")}
    pmc = collections.defaultdict(dict)
    try:
        for ev, pid, val in c.execute("select event_id, pmc_id, value from rocpd_pmc_event"):
            pmc[ev][pmc_names.get(pid, pid)] = pmc[ev].get(pmc_names.get(pid, pid), 0.0) + val
        evmap = {r[0]: r[1] for r in c.execute("select id, event_id from rocpd_kernel_dispatch")}
    except sqlite3.Error:
        evmap = {}
    out = collections.OrderedDict()
    for did, kid, s, e, gx, wx in rows:
        name = sym.get(kid, str(kid))
        if match and match not in name:
            continue
        o = out.setdefault(name, {"n": 0, "ns": [], "grid": gx // max(wx, 1), "wg": wx,
                                  "pmc": collections.defaultdict(float)})
        o["n"] += 1
        o["ns"].append(e - s)
        for k, v in pmc.get(evmap.get(did), {}).items():
            o["pmc"][k] += v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default=None)
    a = ap.parse_args()
    for db in a.dbs:
        print(f"== {db}")
        for name, o in summarize(db, a.match).items():
            ns = o["ns"]
            line = (f"{o['n']:5d} x mean {sum(ns) / len(ns) / 1e3:9.2f} us  min "
                    f"{min(ns) / 1e3:9.2f} us  grid {o['grid']:6d} x {o['wg']:4d}  {name[:90]}")
            print(line)
            for k, v in sorted(o["pmc"].items()):
                print(f"        {k:28s} {v / o['n']:16.1f} per dispatch")


if __name__ == "__main__":
    main()
