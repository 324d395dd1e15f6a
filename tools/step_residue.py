"""Per-step kernel summary of a rocprofv3 --kernel-trace CSV (one replayed step = the kernels
between two consecutive optimizer launches): total kernel time, pio:: share, kernel count, and
the non-pio kernels of the last step.

    python tools/step_residue.py gpurun_out/prof/run_kernel_trace.csv [--marker adamw_kernel]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_kernel")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size", ""))
                for r in rows)
    idx = [i for i, s in enumerate(st) if a.marker in s[2]]
    for k in range(max(1, len(idx) - 3), len(idx)):
        seg = st[idx[k - 1] + 1:idx[k] + 1]
        T = sum((e - b) / 1e3 for b, e, _, _ in seg)
        P = sum((e - b) / 1e3 for b, e, n, _ in seg if "pio::" in n)
        print(f"step: kernel time {T:.1f} us, pio {100 * P / T:.1f}%, span {(seg[-1][1] - seg[0][0]) / 1e3:.1f} us, "
              f"{len(seg)} kernels ({sum(1 for s in seg if 'pio::' not in s[2])} non-pio)")
    seg = st[idx[-2] + 1:idx[-1] + 1]
    t0 = seg[0][0]
    print("non-pio kernels of the last step (start us, duration us, grid, name):")
    for b, e, n, g in seg:
        if "pio::" not in n:
            print(f"{(b - t0) / 1e3:8.1f} {(e - b) / 1e3:6.1f} {g:>8} {n[:100]}")


if __name__ == "__main__":
    main()
