"""Per-kernel summary of rocprofv3 ``--pmc`` passes (``*counter_collection.csv`` under the given
directories): per-dispatch averages of every collected counter and the derived metrics the
reviews ask for.

    python tools/pmc_summary.py gpurun_out/ce/pmc1 gpurun_out/ce/pmc2 [--match ce2_] [--md]

Derived (when the counters are present):
  lds_conflict_pct  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra bank-conflict cycles per LDS-array
                    cycle; falls back to SQ_ACTIVE_INST_LDS when SQ_LDS_IDX_ACTIVE was not collected)
  mfma_util_pct     SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs · CUs · 4 SIMDs)
                    (GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  valu_active_pct   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES      (per-wave share of cycles issuing VALU)
  wait_pct          SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  valu_per_mfma     SQ_INSTS_VALU / SQ_INSTS_MFMA
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(dirs, match):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "")
                if match and match not in name:
                    continue
                c = r["Counter_Name"]
                agg[name][c] += float(r["Counter_Value"])
                cnt[name][c].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(cnt[name][c]))
    out = {}
    for k, d in agg.items():
        out[k] = {c: v / max(1, len(cnt[k][c])) for c, v in d.items()}
    return out


def derived(d, cus):
    x = {}
    den = d.get("SQ_LDS_IDX_ACTIVE") or d.get("SQ_ACTIVE_INST_LDS")
    if den:
        x["lds_conflict_pct"] = 100.0 * d.get("SQ_LDS_BANK_CONFLICT", 0.0) / den
    if d.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
        x["mfma_util_pct"] = 100.0 * d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8.0 * cus * 4)
    if d.get("SQ_WAVE_CYCLES"):
        if d.get("GRBM_GUI_ACTIVE"):  # resident waves per CU, averaged over the dispatch
            x["waves_per_cu"] = d["SQ_WAVE_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8.0 * cus)
        if "SQ_ACTIVE_INST_VALU" in d:
            x["valu_active_pct"] = 100.0 * d["SQ_ACTIVE_INST_VALU"] / d["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_ANY" in d:
            x["wait_pct"] = 100.0 * d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
    if d.get("SQ_INSTS_MFMA"):
        x["valu_per_mfma"] = d.get("SQ_INSTS_VALU", 0.0) / d["SQ_INSTS_MFMA"]
    return x


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args(argv)
    res = load(a.dirs, a.match)
    for k in sorted(res):
        d = res[k]
        x = derived(d, a.cus)
        if a.md:
            print(f"### `{k}`\n")
            print("| metric | per dispatch |\n|---|---:|")
            for c in sorted(x):
                print(f"| **{c}** | {x[c]:.1f} |")
            for c in sorted(d):
                print(f"| {c} | {d[c]:.4g} |")
            print()
        else:
            print(k)
            print("   ", ", ".join(f"{c}={v:.1f}" for c, v in sorted(x.items())))
            print("   ", ", ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))


if __name__ == "__main__":
    main()
