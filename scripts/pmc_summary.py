"""Summarise the rocprofv3 --pmc passes of scripts/pmc_passes.sh into one per-kernel table.

    python scripts/pmc_summary.py gpurun_out/pmc [--top N]

Per kernel (averaged over its dispatches): duration, MFMA busy share of all SIMD cycles
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)), wave-cycle split
(issue-stalled / parked on waitcnt or barrier / issuing), LDS bank-conflict share of LDS
cycles, L2 hit rate, HBM-side bytes fetched / written (FETCH_SIZE / WRITE_SIZE, KiB)."""
import collections
import csv
import glob
import os
import sys


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            k = k.replace("void ", "")[:70]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (f, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    per, dur = load(root)
    avg = lambda xs: sum(xs) / len(xs) if xs else float("nan")  # noqa: E731
    rows = []
    for k, c in per.items():
        g = lambda n: avg(c.get(n, []))  # noqa: E731
        d = avg(dur[k])
        tot = d * len(dur[k])
        # GRBM_GUI_ACTIVE sums the 8 XCDs (calibrated on the 68.7-GFLOP weight-gradient GEMM:
        # MFMA cycles = SQ_INSTS_MFMA x 16 for 16x16x32 bf16 matches this normalisation)
        mfma = g("SQ_VALU_MFMA_BUSY_CYCLES") / max(g("GRBM_GUI_ACTIVE") / 8 * 256 * 4, 1)
        wc = g("SQ_WAVE_CYCLES")
        lds = g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1)
        hit = g("TCC_HIT") / max(g("TCC_HIT") + g("TCC_MISS"), 1)
        rows.append((tot, k, d, mfma, g("SQ_WAIT_INST_ANY") / max(wc, 1),
                     g("SQ_WAIT_ANY") / max(wc, 1), g("SQ_ACTIVE_INST_ANY") / max(wc, 1), lds, hit,
                     g("FETCH_SIZE"), g("WRITE_SIZE"), g("SQ_INSTS_MFMA"), g("SQ_INSTS_VALU")))
    rows.sort(reverse=True)
    print("| kernel | us/dispatch | MFMA busy | wave: issue-stall / parked / issuing | LDS conflict | L2 hit | fetch KiB | write KiB | MFMA insts | VALU insts |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows[:top]:
        tot, k, d, mfma, st, pk, act, lds, hit, fe, wr, nm, nv = r
        print(f"| `{k}` | {d:.1f} | {100*mfma:.1f}% | {100*st:.0f}% / {100*pk:.0f}% / {100*act:.0f}% "
              f"| {100*lds:.2f}% | {100*hit:.0f}% | {fe:.0f} | {wr:.0f} | {nm:.0f} | {nv:.0f} |")


if __name__ == "__main__":
    main()
