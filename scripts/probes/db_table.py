"""Kernel table (count, mean us, total us per step) from one rocprofv3 rocpd SQLite trace.

    python scripts/probes/db_table.py gpurun_out/r6asym2/prof 12
"""
import collections
import glob
import sqlite3
import sys


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    c, t = collections.Counter(), collections.Counter()
    for f in glob.glob(f"{d}/**/*.db", recursive=True):
        for n, s, e in sqlite3.connect(f).execute("select name, start, end from kernels"):
            c[n] += 1
            t[n] += e - s
    print("| kernel | calls | us / call | us / step |\n|---|---|---|---|")
    for n in sorted(t, key=lambda k: -t[k])[:14]:
        short = n.replace("(anonymous namespace)::", "")[:80]
        print(f"| `{short}` | {c[n]} | {t[n] / c[n] / 1e3:.1f} | {t[n] / steps / 1e3:.1f} |")


if __name__ == "__main__":
    main()
