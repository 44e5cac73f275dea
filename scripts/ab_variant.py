#!/usr/bin/env python
"""Build an A/B variant of the native library: the current build with one kernel source
replaced by its version at a git revision (or by another file), for same-box comparisons
with scripts/ab_bench.sh (box-to-box spread of the persistent kernels is 3-8 %).

    python scripts/ab_variant.py <rev-or-path> csrc/lstm2_persist.hip build/ab/old.so
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_char_rnn_amd import _build as B  # noqa: E402


def main(argv):
    src_ref, rel, out = argv
    out = os.path.join(ROOT, out)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    B.build()
    alt = os.path.join(os.path.dirname(out), "variant_" + os.path.basename(rel))
    if os.path.exists(src_ref):
        text = open(src_ref).read()
    else:
        text = subprocess.run(["git", "show", f"{src_ref}:{rel}"], cwd=ROOT, check=True,
                              capture_output=True, text=True).stdout
    with open(alt, "w") as f:
        f.write(text)
    obj = alt + ".o"
    subprocess.run([B._hipcc(), *B.COMMON, "-I", B.CSRC, "-c", alt, "-o", obj], check=True)
    objs = [os.path.join(B.BUILD, os.path.basename(s) + ".o")
            for s in sorted(os.listdir(B.CSRC)) if s.endswith((".hip", ".cpp"))
            and s != os.path.basename(rel)]
    _, ldflags, _ = B._torch_flags()
    subprocess.run([B._hipcc(), *B.COMMON, "-shared", "-o", out, obj, *objs, *ldflags],
                   check=True)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1:])
