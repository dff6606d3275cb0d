"""Summarise rocprofv3 --pmc counter CSVs per kernel (sum over dispatches and the
per-dimension rows), with the derived ratios used in the GEMM notes."""
import collections
import csv
import sys


def load(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dispatches = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"][:80]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dispatches[k].add((p, r["Dispatch_Id"]))
            per[k]["_vgpr"] = float(r.get("VGPR_Count") or 0) + float(r.get("Accum_VGPR_Count") or 0)
            per[k]["_lds"] = float(r.get("LDS_Block_Size") or 0)
    return per, dispatches


def durations(paths):
    """Mean dispatch duration (ns) per kernel from the kernel_trace.csv next to each
    counter CSV (same rocprofv3 run)."""
    import os

    d = collections.defaultdict(list)
    for p in paths:
        kt = os.path.join(os.path.dirname(p), "run_kernel_trace.csv")
        if not os.path.exists(kt):
            continue
        for r in csv.DictReader(open(kt)):
            d[r["Kernel_Name"][:80]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in d.items() if v}


def main(paths):
    per, disp = load(paths)
    dur = durations(paths[:1])
    print("| kernel | counter | value |")
    print("|---|---|---|")
    for k, c in per.items():
        if "gemm" not in k and "mfma" not in k:
            continue
        for name in sorted(c):
            print(f"| `{k}` | {name} | {c[name]:.4g} |")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in c:
                    print(f"| `{k}` | {n}/WAVE_CYCLES | {c[n] / wc:.3f} |")
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            # MFMA busy is summed over SIMDs; GUI_ACTIVE over XCDs (8) -> per-SIMD share
            simds = 256 * 4
            util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * simds)
            print(f"| `{k}` | MFMA busy / (GUI_ACTIVE/8 x 1024 SIMDs) | {util:.3f} |")
        nd = len({d for p_, d in disp[k] if p_ == paths[0]}) or 1
        if c.get("GRBM_GUI_ACTIVE") and k in dur:
            clk = c["GRBM_GUI_ACTIVE"] / nd / 8 / (dur[k] * 1e-9)
            print(f"| `{k}` | mean dispatch ms (profiled) | {dur[k] / 1e6:.3f} |")
            print(f"| `{k}` | effective clock GHz (GUI_ACTIVE/8/duration) | {clk / 1e9:.3f} |")
            if c.get("SQ_INSTS_MFMA"):
                # 16x16x64 i8 MFMA: 16 cycles on one SIMD
                busy = c["SQ_INSTS_MFMA"] / nd * 16 / (1024 * clk * dur[k] * 1e-9)
                print(f"| `{k}` | MFMA pipe occupancy (INSTS_MFMA x 16 cyc / SIMD-cycles) | {busy:.3f} |")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            print(f"| `{k}` | LDS bank conflict / LDS active | "
                  f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f} |")
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m:
            print(f"| `{k}` | L2 hit rate | {h / (h + m):.3f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
