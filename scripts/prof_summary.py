"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a markdown table."""
import sqlite3
import sys


def main(db, title, steps=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"# {title}\n")
    print(f"Source: `{db}` (rocprofv3 --kernel-trace --stats)\n")
    if steps:
        print(f"Kernel time per boosting iteration: {total / 1e6 / steps:.3f} ms over {steps} profiled iterations "
              f"(includes warmup)\n")
    print("| kernel | calls | total ms | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, n, tot, avg, mn, mx in rows:
        short = name.replace("lgap::device::(anonymous namespace)::", "").replace("void ", "")
        short = short.split("(")[0]
        print(f"| `{short[:70]}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | "
              f"{100.0 * tot / total:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "kernel profile",
         int(sys.argv[3]) if len(sys.argv) > 3 else None)
