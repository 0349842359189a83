"""One line per op of a bench.py JSON line (the measured numbers only)."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "check", d.get("check", {}).get("ok"))
keys = ("ms", "kernel_ms", "frac", "local_sort_ms", "reduce_frac", "scan_frac", "graph_ms", "predicted_speedup_8",
        "combine_ms")
for k, v in d.get("ops", {}).items():
    if not isinstance(v, dict):
        continue
    sel = {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items() if kk in keys}
    chk = v.get("check", {})
    print(k, sel, chk.get("ok") if isinstance(chk, dict) else "")
    for sub in ("per_rank_of_8", "flags"):
        if isinstance(v.get(sub), dict):
            print("   ", sub, {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v[sub].items() if kk in keys})
