"""Per-evaluation kernel table from two rocprofv3 kernel traces (rocpd SQLite output) of the
same program run with --runs 0 and --runs N: (N-run counts - 0-run counts) / N per kernel.

    python scripts/probes/kernel_table.py gpurun_out/r6f/prof0 gpurun_out/r6f/prof20 20
"""
import collections
import glob
import re
import sqlite3
import sys


def load(d):
    c, t = collections.Counter(), collections.Counter()
    for f in glob.glob(f"{d}/**/*.db", recursive=True):
        db = sqlite3.connect(f)
        for n, s, e in db.execute("select name, start, end from kernels"):
            c[n] += 1
            t[n] += e - s
    return c, t


def short(n):
    m = re.search(r"d_(\w+?)I[mo]E", n)
    if "k_x3" in n and m:
        return "x3:" + m.group(1)
    if "k_x3" in n and "d_key_refresh" in n:
        return "x3:key_refresh"
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n[:90]


def main():
    d0, dn, runs = sys.argv[1], sys.argv[2], int(sys.argv[3])
    (c0, t0), (cn, tn) = load(d0), load(dn)
    rows, tot_n, tot_t = [], 0.0, 0.0
    for n in cn:
        k = (cn[n] - c0.get(n, 0)) / runs
        us = (tn[n] - t0.get(n, 0)) / runs / 1e3
        if k > 0:
            rows.append((us, k, short(n)))
            tot_n += k
            tot_t += us
    rows.sort(reverse=True)
    print(f"| kernel | dispatches / eval | us / eval |\n|---|---|---|")
    for us, k, n in rows:
        print(f"| `{n}` | {k:.1f} | {us:.1f} |")
    print(f"| **total** | **{tot_n:.1f}** | **{tot_t:.1f}** |")


if __name__ == "__main__":
    main()
