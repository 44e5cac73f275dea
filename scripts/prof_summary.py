"""Summarise a rocprofv3 kernel-trace database (.db) into a per-kernel table (name, calls,
total/avg us, share).

    python scripts/prof_summary.py <dir-or-db> [--top N] [--md] [--grid] [--per-step K]

--grid splits rows by launch geometry (workgroups x threads, VGPR/AGPR counts), which tells the
GEMM shapes apart; --per-step K divides totals by K timed steps."""
import glob
import os
import sqlite3
import sys


def summarize(path, top=30, grid=False):
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"),
                                                      recursive=True)[0]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    key = name_col
    if grid and "grid_x" in cols:
        key = (f"{name_col}, grid_x/workgroup_x, workgroup_x, "
               f"coalesce(vgpr_count,0), coalesce(accum_vgpr_count,0)")
    rows = c.execute(f"select {key}, count(*), sum(end-start), avg(end-start) from kernels "
                     f"group by {key} order by sum(end-start) desc").fetchall()
    tot = sum(r[-2] for r in rows)
    out = []
    for r in rows[:top]:
        n, cnt, s, a = r[0], r[-3], r[-2], r[-1]
        short = n.split("(")[0][:90]
        geo = f"{r[1]}x{r[2]} v{r[3]}+a{r[4]}" if grid and len(r) > 5 else ""
        out.append((short, geo, cnt, s / 1e3, a / 1e3, 100.0 * s / tot))
    return out, tot / 1e3


if __name__ == "__main__":
    p = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    steps = int(sys.argv[sys.argv.index("--per-step") + 1]) if "--per-step" in sys.argv else 0
    rows, tot = summarize(p, top, "--grid" in sys.argv)
    md = "--md" in sys.argv
    unit = "us/step" if steps else "total us"
    div = steps or 1
    if md:
        print(f"| kernel | geometry | calls | {unit} | avg us | share |\n|---|---|---|---|---|---|")
    for name, geo, cnt, s, a, sh in rows:
        if md:
            print(f"| `{name}` | {geo} | {cnt} | {s / div:.1f} | {a:.2f} | {sh:.1f}% |")
        else:
            print(f"{name:<92}{geo:>18}{cnt:>7}{s / div:>12.1f}{a:>10.2f}{sh:>7.1f}%")
    print(f"total kernel time: {tot / div:.1f} {unit}")
