"""Per-(kernel, grid) breakdown of a rocprofv3 kernel trace: separates the calls of one
kernel by launch shape (e.g. self-attention layers vs the encoder cross layer).

    python tools/kernel_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--top 30]
"""
import argparse
import collections
import csv


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv)
    rows = list(csv.DictReader(open(a.trace)))
    d = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-48:]
        key = (name, r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("LDS_Block_Size", "?"))
        d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    print(f"total kernel time {tot / 1e3:.1f} us over {sum(len(v) for v in d.values())} dispatches\n")
    print("| kernel | grid | LDS | calls | avg us | total us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"| `{k[0]}` | {k[1]} | {k[2]} | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {sum(v) / 1e3:.1f} | "
              f"{100 * sum(v) / tot:.1f} |")


if __name__ == "__main__":
    main()
