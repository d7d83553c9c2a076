"""Per-kernel means of every counter of one rocprofv3 --pmc pass (csv output), as csv.

usage: pmc_counters.py <pass dir>

Columns: kernel, dispatches, mean duration (us), then the mean value per dispatch of each counter
in the pass (the pmcx step of scripts/gpu_run.sh). Kernels sorted by total time.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    counters, durations = load(sys.argv[1])
    names = sorted({c for m in counters.values() for c in m})
    rows = []
    for k, m in counters.items():
        d = durations.get(k, [])
        mean = sum(d) / len(d) if d else 0.0
        rows.append((mean * len(d), k, len(d), mean, [sum(m[c]) / len(m[c]) if m.get(c) else 0.0 for c in names]))
    rows.sort(reverse=True)
    print(",".join(["kernel", "dispatches", "mean_us"] + names))
    for _, k, n, mean, vals in rows:
        print(",".join([k.replace(",", ";"), str(n), f"{mean:.2f}"] + [f"{v:.1f}" for v in vals]))


if __name__ == "__main__":
    main()
