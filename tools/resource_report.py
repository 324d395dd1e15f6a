"""Per-kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage remarks.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python tools/resource_report.py remarks.txt [--match substr]
"""
import re
import subprocess
import sys


def parse(path):
    rows, cur = [], None
    for line in open(path):
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        body = m.group(1).strip()
        if body.startswith("Function Name:"):
            cur = {"name": body.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in body:
            k, v = body.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return out[: len(names)]
    except OSError:
        return names


def main():
    path = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    rows = parse(path)
    names = demangle([r["name"] for r in rows])
    print("| kernel | VGPRs | AGPRs | VGPR spill | SGPR spill | scratch B | LDS B | waves/SIMD |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for r, n in zip(rows, names):
        if match not in n:
            continue
        n = re.sub(r"\(.*", "", n)
        print(f"| `{n}` | {r.get('VGPRs', '')} | {r.get('AGPRs', '')} | {r.get('VGPRs Spill', '')} | "
              f"{r.get('SGPRs Spill', '')} | {r.get('ScratchSize [bytes/lane]', '')} | "
              f"{r.get('LDS Size [bytes/block]', '')} | {r.get('Occupancy [waves/SIMD]', '')} |")


if __name__ == "__main__":
    main()
