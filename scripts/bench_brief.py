"""One screen of a bench.py JSON line: headline, roofline and per-leg kernel times."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d.get("value"), "ms", d.get("ms_per_step"), "note", d.get("headline_note"))
r = d.get("roofline") or {}
print("roofline frac", r.get("frac"), "achieved", r.get("achieved"))
for name, v in (d.get("components") or {}).items():
    if not isinstance(v, dict):
        continue
    ks = v.get("kernels") or {}
    print(name, v.get("value"), v.get("ms_per_step"), v.get("error"),
          {k: round(x["avg_ms"], 4) for k, x in ks.items() if isinstance(x, dict) and "avg_ms" in x})
    for sub in ("config4_full_one_gpu", "link_batch", "orphan_remover", "thumbnail_shards",
                "fused_job", "burst"):
        s = v.get(sub)
        if isinstance(s, dict):
            print("  ", sub, s.get("ms_per_step"), s.get("gpu_rep_mismatches"),
                  {k: round(x["avg_ms"], 4) for k, x in (s.get("kernels") or {}).items()
                   if isinstance(x, dict) and "avg_ms" in x})
c = d.get("cpu_baseline") or {}
print("cpu", c.get("value"), c.get("cores"))
