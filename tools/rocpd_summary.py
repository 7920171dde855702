#!/usr/bin/env python3
"""Kernel statistics (and optionally a timeline) from a rocprofv3 SQLite database (the default
output format): python tools/rocpd_summary.py <db> [--timeline FIRST COUNT] [--csv out.csv]"""
import argparse
import csv
import sqlite3


def rows(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    q = f"select {name}, start, end, queue_id, grid_size_x, workgroup_size_x from kernels order by start"
    try:
        return list(con.execute(q))
    except sqlite3.OperationalError:
        q = f"select {name}, start, end, queue_id, grid_x, workgroup_x from kernels order by start"
        return list(con.execute(q))


def short(n):
    return n.replace("void omega::", "").replace("omega::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", nargs=2, type=int, default=None)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    rs = rows(a.db)
    st = {}
    for n, s, e, *_ in rs:
        st.setdefault(short(n), []).append(e - s)
    tot = sum(sum(v) for v in st.values())
    out = []
    for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        out.append((k, len(v), sum(v), sum(v) / len(v), min(v), max(v), 100.0 * sum(v) / tot))
    print(f"{'kernel':48s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}")
    for k, c, t, av, mn, mx, pc in out:
        print(f"{k[:48]:48s} {c:6d} {t / 1e3:10.1f} {av / 1e3:9.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} {pc:6.2f}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            for r in out:
                w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(r[6], 3)])
    if a.timeline:
        first, count = a.timeline
        sel = rs[first:first + count]
        t0 = sel[0][1]
        for n, s, e, q, g, wg in sel:
            print(f"q{q:>3} {short(n)[:34]:34s} grid {g:>8} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}")


if __name__ == "__main__":
    main()
