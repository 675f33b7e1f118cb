"""Parity-bound headroom log: every tolerance-bound GPU test records its measured value next to its bound, so a bound
that a rounding-level change could flip shows up as small headroom (DESIGN.md §5's table is generated from this log,
profiles/r05/parity_margins.jsonl).  Lines go to $GSLM_MARGINS (default gpurun_out/parity_margins.jsonl)."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def record(test, quantity, measured, bound):
    measured, bound = float(measured), float(bound)
    path = os.environ.get("GSLM_MARGINS", os.path.join(ROOT, "gpurun_out", "parity_margins.jsonl"))
    row = {"test": test, "quantity": quantity, "measured": measured, "bound": bound,
           "headroom": (bound / measured) if measured > 0 else None}
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(row) + "\n")
    except OSError:
        pass
    print(f"[margin] {test}: {quantity} = {measured:.3e} (bound {bound:.1e}, headroom {row['headroom'] or 0:.1f}x)")
    return measured
