"""Idle gaps of the GPU kernel timeline in a rocprofv3 kernel-trace database.

usage: prof_gaps.py <db or directory> [min_gap_us]
Prints the distribution of gaps between consecutive kernels (end of one to start of the
next) and the kernels that follow the largest gaps: host round trips show up as gaps
before the first kernel of an iteration.
"""
import glob
import os
import sqlite3
import sys


def short(name):
    n = name.replace("void ", "").replace("lgap::device::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:40]


def main(path, min_gap=3.0):
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True), key=os.path.getsize)[-1]
    c = sqlite3.connect(path)
    rows = sorted(c.execute("select start, end, name from kernels").fetchall())
    # skip the setup phase and the warmup: from the 6th tree's first kernel on
    inits = [i for i, r in enumerate(rows) if "k_f_init" in r[2] or "k_init_tree" in r[2]]
    rows = rows[inits[min(5, len(inits) - 1)]:] if inits else rows
    iters = max(1, len(inits) - 5)
    gaps = {}
    total_gap = 0.0
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        g = (s1 - max(e0, s0)) / 1000.0
        if g < min_gap:
            continue
        key = (short(n0), short(n1))
        cnt, tot = gaps.get(key, (0, 0.0))
        gaps[key] = (cnt + 1, tot + g)
        total_gap += g
    span = (rows[-1][1] - rows[0][0]) / 1000.0
    print(f"span {span:.1f} us over ~{iters} trees, gaps >= {min_gap} us: {total_gap:.1f} us ({100 * total_gap / span:.1f}%)")
    for (a, b), (cnt, tot) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"{tot:10.1f} us {cnt:6d} x {tot / cnt:8.2f} us   {a} -> {b}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 3.0)
