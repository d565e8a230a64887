"""Per-layer conv table of the PRODUCTION schedule from `bench.py --graph-spans FILE` (diagnostic):
    python scripts/spans_table.py SPANS.json [TOP]
Rows: layer, family (conv_fwd / conv_bwd / conv_wgrad ...), calls per step, us per step (the graph-timed call spans,
concurrent calls overlapping), GFLOP, TF/s -- sorted by time, then the family totals."""
import json
import sys
from collections import defaultdict

spans = json.load(open(sys.argv[1]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 60
agg = defaultdict(lambda: [0, 0.0, 0.0])
for s in spans:
    a = agg[(s["layer"], s["family"])]
    a[0] += 1
    a[1] += s["ms"]
    a[2] += s["gflop"]
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
tot = sum(v[1] for _, v in rows)
print(f"{'layer':28s} {'family':11s} calls      us   GFLOP    TF/s")
for (layer, fam), (n, ms, gf) in rows[:top]:
    print(f"{layer:28s} {fam:11s} {n:5d} {ms * 1e3:7.1f} {gf:7.2f} {gf / ms if ms > 0 else 0:7.1f}")
fam = defaultdict(lambda: [0.0, 0.0])
for (layer, f), (n, ms, gf) in rows:
    fam[f][0] += ms
    fam[f][1] += gf
print(f"\nsum of call spans {tot * 1e3:.1f} us")
for f, (ms, gf) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f"  {f:11s} {ms * 1e3:7.1f} us {gf:7.2f} GFLOP {gf / ms if ms > 0 else 0:7.1f} TF/s")
