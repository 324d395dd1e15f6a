"""Summarise a rocprofv3 ``--kernel-trace --stats`` CSV directory into a markdown table.

    python tools/summarize_prof.py gpurun_out/prof [--steps N] > profiles/<name>.md
"""
import argparse
import csv
import glob
import os
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="timed steps in the run (per-step averages)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    stats = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True))
    if not stats:
        sys.exit(f"no *kernel_stats.csv under {a.dir}")
    rows = list(csv.DictReader(open(stats[0])))
    key_t = next(k for k in rows[0] if k.lower().startswith("totaldurationns") or k == "TotalDurationNs")
    tot = sum(float(r[key_t]) for r in rows)
    rows.sort(key=lambda r: -float(r[key_t]))
    print(f"# rocprofv3 kernel stats — {os.path.basename(os.path.normpath(a.dir))}\n")
    print(f"source: `{os.path.relpath(stats[0])}`; total GPU kernel time {tot / 1e6:.3f} ms over all dispatches\n")
    print("| kernel | calls | total ms | avg µs | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[: a.top]:
        name = r.get("Name") or r.get("KernelName") or "?"
        name = name.replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        t = float(r[key_t])
        calls = int(float(r.get("Calls", 0)))
        print(f"| `{name}` | {calls} | {t / 1e6:.3f} | {t / max(calls, 1) / 1e3:.2f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
