"""Kernel gaps of one training step in a rocprofv3 --sys-trace database, with the host API
calls that were running during each gap (is the GPU waiting on the host?).
Usage: systrace_gaps.py run_results.db [marker kernel] [min gap us]"""
import sqlite3
import sys


def main():
    db, marker = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "lstm2_fwd")
    min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    print("tables:", ", ".join(t for t in tabs if not t.startswith("sqlite")))
    ks = list(c.execute("select name, start, end from kernels order by start"))
    idx = [i for i, r in enumerate(ks) if marker in r[0]]
    s, e = idx[-3], idx[-2]
    step = ks[s:e + 1]
    api_tab = next((t for t in ("regions", "hip_api", "rocpd_api", "api") if t in tabs), None)
    cols = []
    if api_tab:
        cols = [r[1] for r in c.execute(f"pragma table_info({api_tab})")]
        print("api table", api_tab, cols[:12])
    t0 = step[0][1]
    for a, b in zip(step, step[1:]):
        gap = (b[1] - a[2]) / 1e3
        print(f"{(a[1] - t0) / 1e3:9.1f} {(a[2] - a[1]) / 1e3:7.1f}  {a[0][:70]}")
        if gap >= min_gap:
            print(f"          gap {gap:6.1f} us before {b[0][:50]}")
            if api_tab and "start" in cols and "end" in cols and "name" in cols:
                rows = list(c.execute(f"select name, start, end from {api_tab} where end > ? and start < ? "
                                      "order by start", (a[2], b[1])))
                for n, st, en in rows[:12]:
                    print(f"             api {(st - t0) / 1e3:9.1f} {(en - st) / 1e3:7.1f}  {str(n)[:60]}")


if __name__ == "__main__":
    main()
