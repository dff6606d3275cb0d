"""Turn a rocprofv3 kernel_stats.csv into a markdown table (committed under profiles/)."""
import csv
import sys


def main(path, title):
    rows = list(csv.DictReader(open(path)))
    print(f"# {title}\n")
    print("| kernel | calls | avg ms | total ms | % |")
    print("|---|---|---|---|---|")
    for r in rows:
        name = r["Name"].replace("|", "\\|")[:90]
        print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
              f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
