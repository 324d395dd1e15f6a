"""Per-launch timeline of ONE replayed training step from a rocprofv3 ``--kernel-trace`` CSV
(the dispatches after the second-to-last optimizer launch): index, kernel, workgroups, threads,
LDS bytes, VGPRs, duration (us) and the gap to the previous kernel.

    python tools/step_timeline.py <kernel_trace.csv> [--marker adamw_kernel]
"""
import argparse
import csv
import re


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_kernel")
    a = ap.parse_args(argv)
    st = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(st) if a.marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("fewer than two optimizer launches in the trace")
    prev = None
    for i, r in enumerate(st[idx[-2] + 1: idx[-1] + 1]):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("pio::", "")[:60]
        wg = 1
        for ax in "XYZ":
            wg *= int(r[f"Grid_Size_{ax}"]) // int(r[f"Workgroup_Size_{ax}"])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{i:3d} {n:60s} wg={wg:6d} thr={r['Workgroup_Size_X']:>4} lds={r['LDS_Block_Size']:>6} "
              f"vgpr={r['VGPR_Count']:>3} {(e - s) / 1e3:7.1f} gap={gap:5.1f}")
        prev = e


if __name__ == "__main__":
    main()
