"""Print value / ms_per_step / roofline frac of bench JSON lines (gpurun_out/bench_<tag>.json)."""
import json
import sys

for tag in sys.argv[1:]:
    try:
        lines = [l for l in open(f"gpurun_out/bench_{tag}.json") if l.startswith("{")]
        d = json.loads(lines[-1])
        print(f"{tag:24s} {d['value']:9.1f} {d['unit']}  {d['ms_per_step']:.3f} ms  frac {d['roofline']['frac']:.4f}")
    except (OSError, IndexError, ValueError, KeyError) as e:
        print(f"{tag:24s} -- {type(e).__name__}: {e}")
