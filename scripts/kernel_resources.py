#!/usr/bin/env python
"""Per-kernel register / spill / LDS table of a HIP source, from the compiler's
kernel-resource-usage remarks (gfx950 device pass only, nothing runs):

    python scripts/kernel_resources.py csrc/lstm2_persist.hip [--filter lstm2_fwd]

A spill inside a persistent kernel's tick loop is a scratch reload with a full vmcnt wait
on the critical path; this is the quick check after every register-pressure change."""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("SGPRs", "sgpr"), ("ScratchSize [bytes/lane]",
          "scratch"), ("VGPRs Spill", "vspill"), ("SGPRs Spill", "sspill"),
          ("LDS Size [bytes/block]", "lds"), ("Occupancy [waves/SIMD]", "occ")]


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names),
                             capture_output=True, text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--filter", default="")
    a = ap.parse_args(argv)
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
               "--offload-device-only", "-c", os.path.abspath(a.source),
               "-I", os.path.join(ROOT, "csrc"), "-Rpass-analysis=kernel-resource-usage",
               "-o", os.path.join(td, "k.o")]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=td)
    if r.returncode != 0:
        print(r.stderr, file=sys.stderr)
        return r.returncode
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
            continue
        if cur is None or ":" not in body:
            continue
        k, v = body.rsplit(":", 1)
        for label, key in FIELDS:
            if k.strip() == label:
                cur[key] = v.strip()
    names = demangle([r_["name"] for r_ in rows])
    keys = [k for _, k in FIELDS]
    print("| kernel | " + " | ".join(keys) + " |")
    print("|---" * (len(keys) + 1) + "|")
    for n, r_ in zip(names, rows):
        if a.filter and a.filter not in n:
            continue
        n = n.split("(")[0]
        print(f"| `{n}` | " + " | ".join(str(r_.get(k, "")) for k in keys) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
