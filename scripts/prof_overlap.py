"""Overlap of collective kernels with compute kernels in a rocprofv3 kernel-trace database.

usage: prof_overlap.py <db or directory> [pattern]
For every kernel whose name contains `pattern` (default "nccl", the RCCL device kernels),
sums the part of its [start, end) interval covered by kernels that do NOT match the
pattern (the learner's compute stream). Prints the totals and the compute kernels the
collectives overlapped with, as a markdown table.
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("lgap::device::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main(path, pat="nccl"):
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True), key=os.path.getsize)[-1]
    c = sqlite3.connect(path)
    rows = sorted(c.execute("select start, end, name from kernels").fetchall())
    coll = [r for r in rows if pat in r[2].lower()]
    comp = [r for r in rows if pat not in r[2].lower()]
    total = sum(e - s for s, e, _ in coll)
    covered = 0
    with_k = defaultdict(float)
    j0 = 0
    for s, e, _ in coll:
        while j0 < len(comp) and comp[j0][1] <= s - 10_000_000:
            j0 += 1
        segs = []
        for cs, ce, cn in comp[j0:]:
            if cs >= e:
                break
            lo, hi = max(s, cs), min(e, ce)
            if hi > lo:
                segs.append((lo, hi))
                with_k[short(cn)] += (hi - lo) / 1e3
        segs.sort()
        cur_lo = cur_hi = None
        for lo, hi in segs:  # union of the overlapping compute intervals
            if cur_hi is None or lo > cur_hi:
                if cur_hi is not None:
                    covered += cur_hi - cur_lo
                cur_lo, cur_hi = lo, hi
            else:
                cur_hi = max(cur_hi, hi)
        if cur_hi is not None:
            covered += cur_hi - cur_lo
    print(f"# Collective / compute overlap (`{os.path.basename(path)}`)\n")
    print(f"{len(coll)} collective kernels matching '{pat}', {total / 1e3:.1f} us in total; "
          f"{covered / 1e3:.1f} us ({100.0 * covered / max(total, 1):.1f}%) overlapped by compute kernels\n")
    print("| compute kernel | overlap us |\n|---|---:|")
    for k, v in sorted(with_k.items(), key=lambda kv: -kv[1])[:12]:
        print(f"| `{k}` | {v:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
