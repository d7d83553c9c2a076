"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a markdown table.

usage: prof_summary.py <db or directory> [title] [profiled_iterations]
Also reports the kernel timeline's busy fraction (union of kernel intervals over
the span from the first kernel start to the last kernel end): a low fraction
means launch / host gaps dominate.
"""
import glob
import os
import sqlite3
import sys


def _find_db(path):
    if os.path.isdir(path):
        dbs = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True), key=os.path.getsize)
        if not dbs:
            raise SystemExit(f"no .db under {path}")
        return dbs[-1]
    return path


def main(path, title, steps=None):
    db = _find_db(path)
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    iv = sorted(c.execute("select start, end from kernels").fetchall())
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (iv[-1][1] - iv[0][0]) if iv else 0
    print(f"# {title}\n")
    print(f"Source: `{db}` (rocprofv3 --kernel-trace --stats)\n")
    if steps:
        print(f"Kernel time per boosting iteration: {total / 1e6 / steps:.3f} ms over {steps} profiled iterations "
              f"(includes warmup)\n")
    if span:
        print(f"Timeline: span {span / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms ({100.0 * busy / span:.1f}%)\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, n, tot, avg, mn, mx in rows:
        short = name.replace("lgap::device::(anonymous namespace)::", "").replace("void ", "")
        short = short.split("(")[0]
        print(f"| `{short[:70]}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | "
              f"{100.0 * tot / total:.1f} |")
    _phases(c)


def _phases(c):
    """roctx phase ranges (ScopedTimer -> roctxRangePushA, rocprofv3 --marker-trace), host wall time."""
    import json

    try:
        rows = c.execute("select extdata, end - start from regions where category like 'MARKER%'").fetchall()
    except sqlite3.OperationalError:
        return
    agg = {}
    for ext, dur in rows:
        try:
            name = json.loads(ext).get("message", "?")
        except (TypeError, ValueError):
            name = "?"
        n, t = agg.get(name, (0, 0))
        agg[name] = (n + 1, t + dur)
    if not agg:
        return
    print("\nroctx phases (host wall time between push and pop; `rocprofv3 --marker-trace`):\n")
    print("| phase | calls | total ms | avg us |")
    print("|---|---:|---:|---:|")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{name}` | {n} | {t / 1e6:.2f} | {t / 1e3 / n:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "kernel profile",
         int(sys.argv[3]) if len(sys.argv) > 3 else None)
