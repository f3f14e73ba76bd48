"""Condense a tools/pmc_round.sh run into profiles/pmc_<tag>.json (per-launch
HBM traffic of the dominant kernel for bench.py's roofline.traffic).

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM): FETCH_SIZE
reports 1/2 of the bytes of wide coalesced streaming reads on gfx950 and other
access widths are uncalibrated, so when the calibration passes of
tools/pmc_r02.sh exist (c1: FETCH_SIZE, c2: WRITE_SIZE of tools/pmc_calib, which
reads / writes a known 8 N^2 bytes with kernel 5's 8-B-per-lane tile pattern)
the factors are measured from them; otherwise FETCH x2, WRITE x1."""
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
ff, wf, calib = 2.0, 1.0, "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); 8-B/lane loads uncalibrated"


def calib_total(path, kname, counter):
    t = 0.0
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            t += float(r["Counter_Value"])
    return t * 1024.0


c1 = glob.glob(root + "/c1/run_counter_collection.csv")
c2 = glob.glob(root + "/c2/run_counter_collection.csv")
if c1 and c2:
    known = 8.0 * 16384 ** 2
    ff = known / calib_total(c1[0], "k_read", "FETCH_SIZE")
    wf = known / calib_total(c2[0], "k_write", "WRITE_SIZE")
    calib = (f"measured on tools/pmc_calib (8-B/lane tile pattern, 2 GiB known): "
             f"FETCH_SIZE x{ff:.4f}, WRITE_SIZE x{wf:.4f}")
# Round 6: the maps are uncached and the workspace cached, so one write factor cannot
# fit the kernel's mixed stores (the uncached calibration counts an 8-B store as a 32-B
# request).  With the cached-map write pass (w0) and the cached-memory calibration (c3):
# the kernel moves the same bytes either way, so its write bytes are w0's, calibrated.
write_per_launch = wf * write / max(n, 1)
w0 = glob.glob(root + "/w0/run_counter_collection.csv")
c3 = glob.glob(root + "/c3/run_counter_collection.csv")
if w0 and c3:
    wf0 = 8.0 * 16384 ** 2 / calib_total(c3[0], "k_write", "WRITE_SIZE")
    w0_tot, w0_disp = 0.0, set()
    for r in csv.DictReader(open(w0[0])):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
            w0_tot += float(r["Counter_Value"]) * 1024.0
            w0_disp.add(r["Dispatch_Id"])
    write_per_launch = wf0 * w0_tot / max(len(w0_disp), 1)
    calib += (f"; writes from the cached-map pass (DYMU_MAP_MEM=0, {len(w0_disp)} dispatches) "
              f"x{wf0:.4f} (cached calibration): uncached 8-B stores count as 32-B requests")
out = {
    "kernel": name, "dispatches": n, "grid": int(sys.argv[4]) if len(sys.argv) > 4 else 16384,
    "fetch_bytes_raw": fetch, "write_bytes": write,
    "traffic_bytes_per_launch": ff * fetch / max(n, 1) + write_per_launch,
    "traffic_bytes_per_launch_raw": (fetch + write) / max(n, 1),
    "fetch_bytes_per_launch": ff * fetch / max(n, 1),
    "write_bytes_per_launch": write_per_launch,
    "correction": calib,
    "counters": {k: v for k, v in tot.items()},
}
json.dump(out, open(f"profiles/pmc_{tag}.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("kernel", "dispatches", "traffic_bytes_per_launch", "traffic_bytes_per_launch_raw")}))
