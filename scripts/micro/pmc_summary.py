"""Summarise a rocprofv3 results database (kernel trace + counters) into one line per dispatch:
kernel, duration and every collected counter.  Usage: pmc_summary.py <dir> [name-filter]."""
import glob
import sqlite3
import sys

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for db in glob.glob(f"{d}/**/*.db", recursive=True):
    c = sqlite3.connect(db)
    names = {r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")}
    rows = list(c.execute("select dispatch_id, name, duration from kernels order by start"))
    ctr = {}
    if "pmc_events" in names:
        cols = [r[1] for r in c.execute("pragma table_info(pmc_events)")]
        q = "select dispatch_id, counter_name, counter_value from pmc_events" if "counter_value" in cols else None
        if q is None:
            print("pmc_events columns:", cols)
        else:
            for did, cn, v in c.execute(q):
                ctr.setdefault(did, {}).setdefault(cn, 0.0)
                ctr[did][cn] += v
    for did, name, dur in rows:
        if filt and filt not in name:
            continue
        cs = " ".join(f"{k}={v:.0f}" for k, v in sorted(ctr.get(did, {}).items()))
        print(f"{name[:40]:40s} {dur / 1000:8.1f} us  {cs}")
