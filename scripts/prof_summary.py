"""Summarise a rocprofv3 kernel-trace database (.db) into a per-kernel table (name, calls,
total/avg us, share).  Usage: python scripts/prof_summary.py <dir-or-db> [--top N] [--md]"""
import glob
import os
import sqlite3
import sys


def summarize(path, top=30):
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "*.db"))[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start) from kernels "
                     f"group by {name_col} order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = []
    for n, cnt, s, a in rows[:top]:
        short = n.split("(")[0][:90]
        out.append((short, cnt, s / 1e3, a / 1e3, 100.0 * s / tot))
    return out, tot / 1e3


if __name__ == "__main__":
    p = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    rows, tot = summarize(p, top)
    md = "--md" in sys.argv
    if md:
        print("| kernel | calls | total us | avg us | share |\n|---|---|---|---|---|")
    for r in rows:
        if md:
            print(f"| `{r[0]}` | {r[1]} | {r[2]:.1f} | {r[3]:.2f} | {r[4]:.1f}% |")
        else:
            print(f"{r[0]:<92}{r[1]:>7}{r[2]:>12.1f}{r[3]:>10.2f}{r[4]:>7.1f}%")
    print(f"total kernel time: {tot:.1f} us")
