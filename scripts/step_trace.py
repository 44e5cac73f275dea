#!/usr/bin/env python
"""Print the kernel sequence of one training step from a rocprofv3 --kernel-trace database:
start offset, duration and grid of every launch between two consecutive launches of a marker
kernel (default: the two-layer forward).  Usage: step_trace.py run_results.db [marker] [nth]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "lstm2_fwd"
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else -3
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels "
                          "order by start"))
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    s, e = idx[nth], idx[nth + 1]
    t0 = rows[s][1]
    tot = 0.0
    for r in rows[s:e]:
        d = (r[2] - r[1]) / 1e3
        tot += d
        print(f"{(r[1] - t0) / 1e3:9.1f} {d:7.1f} {r[3] // max(r[5], 1):>5}x{r[4]:<3} {r[0][:96]}")
    print(f"launches: {e - s}   kernel time: {tot:.1f} us   span: {(rows[e][1] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
