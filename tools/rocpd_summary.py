"""Kernel-time summary of a rocprofv3 rocpd database (``-d DIR -o run`` → DIR/run_results.db).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--top 40] [--step-of pio::adamw]

Prints per-kernel totals (calls, total/avg µs, share) and, with ``--step-of NAME``, the ordered
kernel sequence of one step (between the last two launches of NAME).
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--step-of", default=None)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tot, n = c.execute("select sum(end-start)/1000.0, count(*) from kernels").fetchone()
    print(f"total kernel time {tot:.1f} us over {n} dispatches")
    rows = c.execute("select name, count(*), sum(end-start)/1000.0, avg(end-start)/1000.0 from kernels "
                     "group by name order by 3 desc limit ?", (a.top,)).fetchall()
    div = max(1, a.steps)
    for name, cnt, s, avg in rows:
        print(f"{s / div:10.1f} us {cnt / div:7.1f}x {avg:8.1f} {100 * s / tot:5.1f}%  {name[:100]}")
    if a.step_of:
        seq = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
        idx = [i for i, r in enumerate(seq) if r[0].startswith(a.step_of)]
        if len(idx) >= 2:
            lo, hi = idx[-2], idx[-1]
            t0 = seq[lo][2]
            for r in seq[lo + 1:hi + 1]:
                print(f"{(r[1] - t0) / 1000:8.1f} {(r[2] - r[1]) / 1000:7.1f}  g=({r[3]},{r[4]},{r[5]})/{r[6]}  {r[0][:90]}")


if __name__ == "__main__":
    main()
