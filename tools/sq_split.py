"""Stall split of GEMM launches from rocprofv3 --pmc counter CSVs (tools/gemm_sq_split.sh): per kernel
instance and grid, the wave-cycle shares issuing (SQ_ACTIVE_INST_ANY), waiting on s_waitcnt / barriers
(SQ_WAIT_ANY) and issue-stalled (SQ_WAIT_INST_ANY) out of SQ_WAVE_CYCLES, the VALU / LDS issue shares,
and MFMA busy per SIMD-cycle (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE / 8).
Usage: python tools/sq_split.py counter_collection.csv [more.csv ...] [--json out.json]"""
import collections
import csv
import json
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"^(?:void )?(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out in args:
        args.remove(out)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in args:
        seen = set()
        for r in csv.DictReader(open(f)):
            k = (short(r["Kernel_Name"]), r.get("Grid_Size", "?"))
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            d = (r.get("Dispatch_Id"), k)
            if d not in seen:
                seen.add(d)
                n[(f, k)] += 1
    res = {}
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVE_CYCLES")
        if not w or "gemm" not in k[0]:
            continue
        row = {"kernel": k[0], "grid": k[1]}
        for name, key in (("issuing", "SQ_ACTIVE_INST_ANY"), ("waitcnt_barrier", "SQ_WAIT_ANY"),
                          ("issue_stalled", "SQ_WAIT_INST_ANY"), ("valu_issue", "SQ_ACTIVE_INST_VALU"),
                          ("lds_issue", "SQ_ACTIVE_INST_LDS"), ("lds_wait", "SQ_WAIT_INST_LDS"),
                          ("vmem_issue", "SQ_ACTIVE_INST_VMEM"), ("salu_issue", "SQ_ACTIVE_INST_SCA")):
            if key in c:
                row[name] = round(c[key] / w, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            row["mfma_busy_per_simd_cycle"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 3)
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SALU"):
            if key in c:
                row[key] = c[key]
        res[f"{k[0]} grid {k[1]}"] = row
        print(json.dumps(row))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
