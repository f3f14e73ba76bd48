"""Sum rocprofv3 --pmc counter_collection CSVs per counter for one kernel."""
import csv, glob, sys, collections
root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_fim_pass"
tot = collections.Counter(); disp = collections.defaultdict(set); dur = {}
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k, v in sorted(tot.items()):
    print(f"{k:24s} {v:.4e}  dispatches={len(disp[k])}")
