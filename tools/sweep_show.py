"""Summarise a tools/sweep.sh log: per setting, the second solve's wall time, passes and visits."""
import json
import sys

cur = None
for line in open(sys.argv[1]):
    if line.startswith("v "):
        cur = line[2:].strip()
        continue
    try:
        d = json.loads(line)
    except ValueError:
        continue
    r = d["runs"]
    ms = [x["wall_s"] * 1e3 for x in r]
    print(f"N={d['N']:<6d} {cur:48s} ms {min(ms[:2]):7.2f} ({ms[0]:.2f} {ms[1]:.2f}) passes {r[1]['passes']:5d} "
          f"visits {r[1]['tile_visits']:8d} sweeps/visit {r[1]['inner_sweeps'] / max(1, r[1]['tile_visits']):.2f}")
