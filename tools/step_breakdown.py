"""Kernel-time breakdown of ONE replayed training step from a rocprofv3 ``--kernel-trace`` CSV:
the dispatches between the last two optimizer launches, grouped by kernel (template arguments
kept), as a markdown table.

    python tools/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--marker adamw_kernel]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)  # drop the parameter list
    name = name.replace("void ", "")
    return name[:90]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_kernel")
    a = ap.parse_args(argv)
    rows = list(csv.DictReader(open(a.trace)))
    st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    idx = [i for i, s in enumerate(st) if a.marker in s[2]]
    if len(idx) < 2:
        raise SystemExit("fewer than two optimizer launches in the trace")
    step = st[idx[-2] + 1: idx[-1] + 1]
    span = (step[-1][1] - step[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in step) / 1e3
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, n in step:
        agg[short(n)][0] += 1
        agg[short(n)][1] += (e - s) / 1e3
    print(f"one step: {len(step)} kernels, kernel time {busy:.1f} us, span {span:.1f} us\n")
    print("| kernel | launches | us | % |")
    print("|---|---:|---:|---:|")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{n}` | {c} | {t:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    main()
