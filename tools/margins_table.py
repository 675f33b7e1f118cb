"""DESIGN.md §5's parity headroom table from the margin logs tests/margins.py writes.

    python tools/margins_table.py LOG.jsonl [--perturbed PERTURBED.jsonl]

One row per (test, quantity) with the parametrised cases folded together (test[a], test[b] -> test): the worst
(largest) measured value over the cases, the bound, and the headroom bound / measured.  With --perturbed, the same
quantity's worst value in a second log (a run of a deliberately perturbed build, e.g. one extra rounding in the
exponent) goes beside it: a bound that holds there too measures correctness, not one build's rounding."""
import argparse
import json
import re


def load(path):
    rows = {}
    for line in open(path):
        line = line.strip()
        if not line:
            continue
        r = json.loads(line)
        key = (re.sub(r"\[.*\]$", "", r["test"]), r["quantity"])
        m, b = float(r["measured"]), float(r["bound"])
        old = rows.get(key)
        if old is None or m > old[0]:
            rows[key] = (m, b)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--perturbed")
    a = ap.parse_args()
    base = load(a.log)
    pert = load(a.perturbed) if a.perturbed else {}
    hdr = "| test | quantity | bound | measured (worst case) | headroom |"
    sep = "|---|---|---|---|---|"
    if pert:
        hdr += " perturbed build |"
        sep += "---|"
    print(hdr)
    print(sep)
    for (t, q), (m, b) in sorted(base.items(), key=lambda kv: (kv[1][1] / kv[1][0]) if kv[1][0] > 0 else 1e30):
        head = f"{b / m:.0f}x" if m > 0 else "exact"
        row = f"| `{t}` | {q} | {b:.3g} | {m:.2e} | {head} |"
        if pert:
            pm = pert.get((t, q))
            row += (f" {pm[0]:.2e} |" if pm else " -- |")
        print(row)


if __name__ == "__main__":
    main()
