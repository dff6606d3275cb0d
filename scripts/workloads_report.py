"""Markdown tables of the reference workloads from the JSONL files that
scripts/gpu_check.sh writes (dots / logreg, eager and hipGraph replay)."""
import json
import sys


def load(path):
    try:
        return [json.loads(line) for line in open(path) if line.strip()]
    except FileNotFoundError:
        return []


def main(out_dir="gpurun_out"):
    dots = load(f"{out_dir}/dots.jsonl")
    dotsg = {(d["mode"], d["k"], d["n"]): d for d in load(f"{out_dir}/dots_graphs.jsonl")}
    print("## Replicated dot products, fixed(8,27) over Z_2^128 -- seconds per evaluation\n")
    print("Stacked 3-party session on one MI355X (LocalMooseRuntime), mean of 3 evaluations "
          "after a warm-up; reference = BASELINE.md (3 gRPC workers on c5.9xlarge).\n")
    print("| mode | k | n | eager (s) | hipGraph (s) | reference (s) | speedup (best) |")
    print("|---|---|---|---|---|---|---|")
    for d in dots:
        g = dotsg.get((d["mode"], d["k"], d["n"]))
        best = min(d["seconds_mean"], g["seconds_mean"]) if g else d["seconds_mean"]
        ref = d.get("reference_s")
        print(f"| {d['mode']} | {d['k']} | {d['n']} | {d['seconds_mean']:.5f} | "
              f"{g['seconds_mean']:.5f} |" if g else
              f"| {d['mode']} | {d['k']} | {d['n']} | {d['seconds_mean']:.5f} | - |", end="")
        print(f" {ref} | {ref / best:.1f}x |" if ref else " - | - |")
    lr = load(f"{out_dir}/logreg.jsonl")
    lrg = {(d["batch_size"], d["n_iter"]): d for d in load(f"{out_dir}/logreg_graphs.jsonl")}
    print("\n## LogReg training (100 features, fixed(24,40), SGD + momentum) -- seconds per run\n")
    print("| batch | iters | eager (s) | hipGraph (s) | reference (s) | speedup (best) |")
    print("|---|---|---|---|---|---|")
    for d in lr:
        key = (d["batch_size"], d["n_iter"])
        g = lrg.get(key)
        mean = d["session_s"]["mean"]
        gm = g["session_s"]["mean"] if g else None
        best = min(mean, gm) if gm else mean
        ref = d.get("reference_s")
        print(f"| {key[0]} | {key[1]} | {mean:.3f} | {gm:.3f} |" if gm else
              f"| {key[0]} | {key[1]} | {mean:.3f} | - |", end="")
        print(f" {ref} | {ref / best:.1f}x |" if ref else " - | - |")


if __name__ == "__main__":
    main(*sys.argv[1:])
