#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (usage: bench_summary.py <bench.json> ...)."""
import json, sys
for path in sys.argv[1:]:
    d = json.load(open(path))
    r = d["roofline"]
    print(f"== {path}\nC2 value {d['value']:.0f} outer/s, {d['ms_per_step']} ms/step, kernel {r['kernel_ms']} ms, "
          f"frac {r['frac']}, traffic {r.get('traffic')}")
    c3 = d.get("c3_mintime_plus_mincurv", {})
    print(f"C3 wall {c3.get('wall_ms_mean')} ms (mc {c3.get('kernel_ms_mincurv')} / mt {c3.get('kernel_ms_mintime')})")
    c4 = d.get("c4_sweep_7tracks_x_512", {})
    print(f"C4 {c4.get('ms')} ms, {c4.get('tracks_per_s')} tracks/s, lapΔ {c4.get('lap_delta_vs_oracle', {}).get('max_abs_s')}")
    c5 = d.get("c5_oval_n10000", {})
    print(f"C5 {c5.get('kernel_ms')} ms, frac {c5.get('roofline', {}).get('frac')}; C5 min-time {c5.get('mintime', {}).get('kernel_ms')} ms")
    o = d.get("open_mode_n2000", {})
    print(f"open mc {o.get('kernel_ms_mincurv')} mt {o.get('kernel_ms_mintime')}, vs oracle {o.get('vs_oracle', {}).get('evals_equal')}")
    p = d.get("c2_pcie_inclusive", {})
    print(f"C2 PCIe call {p.get('call_ms_median')} ms ({p.get('outer_iters_per_s')}/s), abi {p.get('abi_call_ms_median')}")
    dr = d.get("dropin_b1_latency", {})
    if dr:
        ov = [v.get("mincurv_abi_overhead_ms") for v in dr.values()]
        print(f"drop-in B=1 overhead ms {min(ov)}..{max(ov)}; cmap1 n2000 mc {dr.get('cmap1_n2000', {}).get('mincurv_ms')}")
    cb = d.get("cpu_baseline") or {}
    print(f"cpu baseline {cb.get('value')} {cb.get('kind')}")
