"""Per-pass analysis of a rocprofv3 kernel trace (development tool)."""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_fim_pass" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
n = len(d)
print("launches", n, "total_ms %.1f" % (sum(d) / 1e3))
# assume the last solve is the final len/solves launches; print deciles of the last solve
solves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
per = n // solves
last = d[-per:]
import statistics
print("per-solve launches", per, "sum_ms %.1f" % (sum(last) / 1e3), "median_us %.1f" % statistics.median(last))
for q in range(10):
    seg = last[q * per // 10:(q + 1) * per // 10]
    print("decile %d: n=%d sum_ms=%.1f mean_us=%.1f max_us=%.1f" % (q, len(seg), sum(seg) / 1e3, sum(seg) / len(seg), max(seg)))
