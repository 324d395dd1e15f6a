"""One-line-per-kernel table of the derived PMC metrics (tools/pmc_summary.py), kernels ranked by
their share of SQ_WAVE_CYCLES.

    python tools/pmc_table.py gpurun_out/pmc_mlm/p1 gpurun_out/pmc_mlm/p2 [--top 16] [--match pio::]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as ps  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=16)
    ap.add_argument("--match", default="pio::")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args(argv)
    res = ps.load(a.dirs, a.match)
    rows = sorted(((d.get("SQ_WAVE_CYCLES", 0.0), k, d, ps.derived(d, a.cus)) for k, d in res.items()), reverse=True)
    print("| kernel | waves | waves / CU (mean resident) | MFMA busy % | VALU active % (per wave) | wait % | LDS bank-conflict % | VALU / MFMA instr |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for _, k, d, x in rows[:a.top]:
        print(f"| `{k[:72]}` | {d.get('SQ_WAVES', 0):.0f} | {x.get('waves_per_cu', 0):.1f} | {x.get('mfma_util_pct', 0):.1f} | "
              f"{x.get('valu_active_pct', 0):.1f} | {x.get('wait_pct', 0):.1f} | {x.get('lds_conflict_pct', 0):.1f} | "
              f"{x.get('valu_per_mfma', 0):.1f} |")


if __name__ == "__main__":
    main()
