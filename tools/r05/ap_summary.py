"""One line per tools/alloc_probe.py log: per-pass k_onesweep ms (min / mean / max) over its sorts."""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
passes = [p for r in rows if "passes" in r for p in r["passes"] if p > 0]
sorts = [r["ms"] for r in rows if "ms" in r]
ok = all(r.get("verified", True) for r in rows)
if passes:
    print(f"pass ms {min(passes):.3f} / {sum(passes) / len(passes):.3f} / {max(passes):.3f}  "
          f"sorts {' '.join(f'{s:.2f}' for s in sorts)}  verified {ok}")
else:
    print("no passes recorded")
