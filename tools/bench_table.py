#!/usr/bin/env python3
"""One line per committed bench JSON (profiles/<tag>_bench.json): the numbers DESIGN.md quotes."""
import json
import sys

for f in sys.argv[1:]:
    r = json.load(open(f))
    cb, dyn, rf = r.get("cpu_baseline") or {}, r.get("dynamic") or {}, r["roofline"]
    print(f"{f}: value {r['value']:.3g} {r['unit']} | ms/step {r['ms_per_step']:.3f} | p50 frame {r['p50_frame_ms']:.3f} ms"
          f" | dynamic {dyn.get('ms_per_step_dynamic', float('nan')):.3f} ms, rebuild frame {dyn.get('p50_frame_ms_rebuild', float('nan')):.3f} ms"
          f" | frac {rf['frac']:.4f} single-issue {rf['single_issue']['frac']:.3f} equivalent {rf['equivalent']['frac']:.3f}"
          f" | traffic {rf['traffic']} | kernel_ms {r['kernel_ms']}"
          f" | cpu {cb.get('value', float('nan')):.3g} on {cb.get('cores')} thr, 1 thr {cb.get('one_thread', {}).get('value', float('nan')):.3g}")
