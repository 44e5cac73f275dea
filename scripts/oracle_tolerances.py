"""Summarise a DCR_ORACLE_LOG file (tests/oracle.py): per test key, the largest measured relative
and row-block errors over every parametrisation and parameter, where they occurred, the
tolerance in force and twice the measured maximum (the tolerance rule of tests/oracle.py).

    python scripts/oracle_tolerances.py gpurun_out/<run>/oracle.jsonl > profiles/r4_oracle_errors.md
"""
import json
import re
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from oracle import TOL  # noqa: E402


def main(path):
    rows = [json.loads(line) for line in open(path) if line.strip()]
    by = {}
    for r in rows:
        k = r["key"]
        if k == "native_model" and re.search(r"[\[-]nas[\]-]", r["test"]):  # (pre-split logs)
            k = "native_model_nas"
        by.setdefault(k, []).append(r)
    print(f"# Oracle gradient errors ({len(rows)} parameter comparisons)\n")
    print("| key | cases | max rel | at | max blk | at | tol (rel, blk) | 2x measured |")
    print("|---|---|---|---|---|---|---|---|")
    for k in sorted(by):
        rs = by[k]
        mr = max(rs, key=lambda r: r["rel"])
        mb = max(rs, key=lambda r: r["blk"])
        short = lambda r: f"{r['test'].split('::')[-1].split(' ')[0]} {r['param']}"  # noqa: E731
        t = TOL.get(k, ("?", "?"))
        print(f"| {k} | {len(set(r['test'] for r in rs))} | {mr['rel']:.2e} | {short(mr)} | "
              f"{mb['blk']:.2e} | {short(mb)} | {t[0]}, {t[1]} | "
              f"{2 * mr['rel']:.1e}, {2 * mb['blk']:.1e} |")


if __name__ == "__main__":
    main(sys.argv[1])
