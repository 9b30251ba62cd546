import json, sys
for l in sys.stdin:
    try:
        d = json.loads(l)
    except Exception:
        continue
    print(d["workload"], d["ranks"], "r" + str(d.get("rank", 0)), d["inflight"], d.get("mode"), d.get("events"), d.get("cumask"), "gather" if d.get("gather") else "", "B" + str(d.get("batch", 1)),
          round(d["ms_per_frame"], 3), round(d["gsteps"], 2))
