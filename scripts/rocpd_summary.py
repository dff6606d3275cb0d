"""Kernel table from a rocprofv3 SQLite result (``run_results.db``), as markdown.

    python scripts/rocpd_summary.py A.db [B.db --per N] [--title T]

With one database: calls, average and total time per kernel.  With two (the same program
run with k and k + N evaluations), the per-evaluation difference B - A divided by N --
the kernels of ONE evaluation, warm-ups and setup subtracted out.  Also prints the
timeline span of the last ``--per`` dispatch groups' kernels (busy vs. wall)."""
import argparse
import collections
import sqlite3


def load(path):
    c = sqlite3.connect(path)
    names = {r[0]: r[1] for r in c.execute(
        "select id, coalesce(display_name, kernel_name) from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end, queue_id from rocpd_kernel_dispatch "
                     "order by start").fetchall()
    return [(names.get(k, str(k)), s, e, q) for k, s, e, q in rows]


def stats(rows):
    acc = collections.OrderedDict()
    for n, s, e, _ in rows:
        a = acc.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    return acc


def short(n, w=80):
    return n.replace("(anonymous namespace)::", "").replace("|", "\\|")[:w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b", nargs="?")
    ap.add_argument("--per", type=int, default=1)
    ap.add_argument("--title", default="kernels")
    a = ap.parse_args()
    A = stats(load(a.a))
    print(f"# {a.title}\n")
    if a.b is None:
        tot = sum(v[1] for v in A.values())
        print("| kernel | calls | avg us | total ms | % |\n|---|---|---|---|---|")
        for n, (k, t) in sorted(A.items(), key=lambda kv: -kv[1][1]):
            print(f"| `{short(n)}` | {k} | {t / k / 1e3:.2f} | {t / 1e6:.3f} | "
                  f"{100 * t / tot:.1f} |")
        return
    rows_b = load(a.b)
    B = stats(rows_b)
    diff = []
    for n, (k, t) in B.items():
        k0, t0 = A.get(n, (0, 0))
        dk, dt = (k - k0) / a.per, (t - t0) / a.per
        if dk > 0.01:
            diff.append((n, dk, dt))
    diff.sort(key=lambda x: -x[2])
    tot = sum(d[2] for d in diff)
    calls = sum(d[1] for d in diff)
    print(f"Per evaluation ({a.per} evaluations difference): {calls:.1f} kernel dispatches, "
          f"{tot / 1e3:.1f} us of kernel time.\n")
    print("| kernel | calls / eval | avg us | us / eval | % |\n|---|---|---|---|---|")
    for n, dk, dt in diff:
        print(f"| `{short(n)}` | {dk:.1f} | {dt / dk / 1e3:.2f} | {dt / 1e3:.1f} | "
              f"{100 * dt / tot:.1f} |")


if __name__ == "__main__":
    main()
