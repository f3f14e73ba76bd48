"""Condense a tools/pmc_round.sh run into profiles/pmc_<tag>.json (per-launch
HBM traffic of the dominant kernel for bench.py's roofline.traffic).

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM): FETCH_SIZE
reports 1/2 of the bytes of wide coalesced streaming reads on gfx950, so it is
doubled here; other access widths are uncalibrated there (our loads are 8 B
per lane), which is why the raw value is kept beside the corrected one."""
import csv, glob, json, sys, collections
root, tag = sys.argv[1], sys.argv[2]
kern = sys.argv[3] if len(sys.argv) > 3 else "k_fim_pass"
tot = collections.Counter(); disp = collections.defaultdict(set); name = None
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
n = len(disp["FETCH_SIZE"])
fetch = tot["FETCH_SIZE"] * 1024.0
write = tot["WRITE_SIZE"] * 1024.0
out = {
    "kernel": name, "dispatches": n, "grid": int(sys.argv[4]) if len(sys.argv) > 4 else 16384,
    "fetch_bytes_raw": fetch, "write_bytes": write,
    "traffic_bytes_per_launch": (2.0 * fetch + write) / max(n, 1),
    "traffic_bytes_per_launch_raw": (fetch + write) / max(n, 1),
    "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); 8-B/lane loads uncalibrated",
    "counters": {k: v for k, v in tot.items()},
}
json.dump(out, open(f"profiles/pmc_{tag}.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("kernel", "dispatches", "traffic_bytes_per_launch", "traffic_bytes_per_launch_raw")}))
