"""In-tree native build: compiles ``csrc/*.hip`` (device kernels, gfx950 only) and
``csrc/*.cpp`` (torch op bindings) with ``hipcc`` and links them into
``distributed_char_rnn_amd/_C.so``.

No hipify, no JIT cache, no CUDA path: the library is built for ``--offload-arch=gfx950`` and
loaded with ``torch.ops.load_library`` (see ``ops/native.py``).  Objects are cached under
``build/`` and rebuilt when the source or any ``csrc/*.h`` header is newer.  The library's
sidecar ``_C.so.srchash`` records the sha256 of every ``csrc/`` file plus the compile flags it
was built from; the loader compares it with the sources it finds next to it and rebuilds (or,
with ``DCR_AUTOBUILD=0``, refuses to load) a library that does not match them.

Usage: ``python -m distributed_char_rnn_amd._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
OUT = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("DCR_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = os.path.join(rocm, "bin", "hipcc")
    if os.path.exists(cand):
        return cand
    found = shutil.which("hipcc")
    if not found:
        raise RuntimeError("hipcc not found: set ROCM_PATH")
    return found


def _cxx() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    clang = os.path.join(rocm, "lib", "llvm", "bin", "clang++")  # understands __bf16 on x86
    return os.environ.get("DCR_CXX", clang if os.path.exists(clang) else "c++")


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-I{sysconfig.get_paths()['include']}",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    ldflags = [f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               f"-Wl,-rpath,{torch_lib}"]
    return cflags, ldflags, libdirs


COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
          "-ffp-contract=fast"]
# per-kernel register / scratch report of every device compile (parsed into _C.resources.json)
DEV_FLAGS = ["-Rpass-analysis=kernel-resource-usage"]
RESOURCES = os.path.join(PKG_DIR, "_C.resources.json")
# Sources whose kernels spin on each other across workgroups (persistent hand-offs, in-launch
# waits).  None of their kernels may spill to scratch: at the register limit this compiler has
# reloaded a spilled 128-bit MFMA fragment without one of its dwords (round 6, docs/STATUS.md:
# the wide BPTT's steady tick body with wide_pf=0 computed NaN gradients), and a wrong value
# in a hand-off index is a spin timeout, not a wrong number.  The build fails instead (except
# for KNOWN_SPILLS).
NO_SPILL_SOURCES = ("lstm2_persist.hip", "lstm2_bwd_wide.hip", "lstm2_bwd_rs.hip",
                    "lstm_persist.hip", "lstm_persist_nt.hip", "gru_persist.hip",
                    "generate.hip", "tail.hip")
# instantiations that spilled before the guard existed (all covered by the GPU oracle tests;
# none is on the headline path): the two-layer dropout forward at H = 512 with 3-4 row groups per
# workgroup (lstm2_persist.hip KS = 4, G >= 3, DROP: B > 512 with dropout) and the stamped (DIAG)
# NT forward instantiations.  (Round 6 removed four: the G = 2 forward no longer double-buffers
# its payload at KS = 4 -- spill-free and 4 % faster at B = 512 -- and the never-launched
# fused-input single-layer forwards at KS = 6 / 8 are no longer instantiated.)
KNOWN_SPILLS = frozenset({
    "_ZN3dcr24lstm2_fwd_persist_kernelILi4ELi3ELb1ELb0ELb0EEEvNS_9Lstm2ArgsE",
    "_ZN3dcr24lstm2_fwd_persist_kernelILi4ELi4ELb1ELb0ELb0EEEvNS_9Lstm2ArgsE",
    "_ZN3dcr26lstm_fwd_persist_nt_kernelILi16ELi2ELb1ELb0EEEvNS_11PersistArgsE",
    "_ZN3dcr26lstm_fwd_persist_nt_kernelILi16ELi4ELb1ELb0EEEvNS_11PersistArgsE",
})


def parse_resource_remarks(text: str) -> dict:
    """``-Rpass-analysis=kernel-resource-usage`` output -> {kernel: {field: int}}."""
    import re

    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return out


def source_hash() -> str:
    """sha256 over every csrc/ file (name + bytes), the compile flags and the target arch."""
    import hashlib

    h = hashlib.sha256()
    h.update(" ".join(COMMON + DEV_FLAGS).encode())
    for f in sorted(glob.glob(os.path.join(CSRC, "*"))):
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode() + b"\0")
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def recorded_hash(lib: str = OUT) -> str | None:
    try:
        with open(lib + ".srchash") as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def _stale(obj: str, src: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    if os.path.getmtime(src) > t:
        return True
    return any(os.path.getmtime(h) > t for h in headers)


class _BuildLock:
    """Inter-process lock around a build: the ranks of a multi-process run that all find a
    stale library would otherwise compile into the same object files and link into the same
    temporary library at once (one rank then loads a half-written _C.so)."""

    def __enter__(self):
        import fcntl

        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        self.fh = open(OUT + ".lock", "w")
        fcntl.flock(self.fh, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self.fh, fcntl.LOCK_UN)
        self.fh.close()


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    with _BuildLock():
        return _build_locked(force, jobs, verbose)


def _build_locked(force: bool, jobs: int | None, verbose: bool) -> str:
    os.makedirs(BUILD, exist_ok=True)
    want = source_hash()
    if not force and recorded_hash() == want and os.path.exists(OUT):
        return OUT  # another process built it while this one waited for the lock
    if recorded_hash() != want and os.path.exists(OUT):
        force = True  # the library was built from other sources (mtimes can lie after a copy)
    hipcc = _hipcc()
    cflags, ldflags, _ = _torch_flags()
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    dev_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    host_srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    jobs = min(jobs, 16)

    def compile_one(src: str):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        res = obj + ".res.json"
        if not force and not _stale(obj, src, headers) and (src.endswith(".cpp") or
                                                              os.path.exists(res)):
            return obj, None
        if src.endswith(".hip"):
            cmd = [hipcc, *COMMON, *DEV_FLAGS, "-I", CSRC, "-c", src, "-o", obj]
        else:  # torch bindings: host-only C++ (no device code), compiled by the host compiler
            cmd = [_cxx(), "-O2", "-std=c++17", "-fPIC", "-I", CSRC, *cflags, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
        if src.endswith(".hip"):
            import json

            with open(res, "w") as fh:
                json.dump({"source": os.path.basename(src),
                           "kernels": parse_resource_remarks(r.stderr)}, fh)
        return obj, None

    with ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(compile_one, dev_srcs + host_srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("native build failed:\n" + "\n\n".join(errs))
    objs = [o for o, _ in results]
    _check_resources(dev_srcs)
    if force or not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT)
                                               for o in objs):
        tmp = f"{OUT}.tmp{os.getpid()}"
        cmd = [hipcc, *COMMON, "-shared", "-o", tmp, *objs, *ldflags]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
    tmp_hash = f"{OUT}.srchash.tmp{os.getpid()}"
    with open(tmp_hash, "w") as fh:
        fh.write(want + "\n")
    os.replace(tmp_hash, OUT + ".srchash")
    return OUT


def _check_resources(dev_srcs) -> None:
    """Collect the per-kernel reports into _C.resources.json; fail on a spilling kernel of a
    NO_SPILL_SOURCES file."""
    import json

    table, bad = {}, []
    for src in dev_srcs:
        with open(os.path.join(BUILD, os.path.basename(src) + ".o.res.json")) as fh:
            rep = json.load(fh)
        table[rep["source"]] = rep["kernels"]
        if rep["source"] in NO_SPILL_SOURCES:
            for k, v in rep["kernels"].items():
                if (v.get("ScratchSize", 0) or v.get("VGPRs Spill", 0)) and k not in KNOWN_SPILLS:
                    bad.append(f"{rep['source']}: {k} scratch {v.get('ScratchSize')} B/lane, "
                               f"{v.get('VGPRs Spill')} VGPRs spilled")
    with open(RESOURCES, "w") as fh:
        json.dump(table, fh, indent=0, sort_keys=True)
    if bad:
        raise RuntimeError("persistent kernels must not spill (see _build.NO_SPILL_SOURCES):\n"
                           + "\n".join(bad))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
