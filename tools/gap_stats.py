"""Idle gaps between pass launches in a rocprofv3 kernel trace (development tool).

usage: python3 tools/gap_stats.py <run_kernel_trace.csv> [solves]

Splits the pass-kernel launches into solves at gaps above 300 us (the bench's
between-solve host work) and reports per solve: launches, summed kernel time,
span, and the idle time between launches split into small (<= 10 us) and large
gaps (the host round trips of the convergence checks).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = [r for r in csv.DictReader(open(path)) if "fim_pass" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    solves, cur = [], [0]
    for i in range(1, len(st)):
        if (st[i] - en[i - 1]) / 1e3 > 300:
            solves.append(cur)
            cur = []
        cur.append(i)
    solves.append(cur)
    for s in solves:
        dur = sum(en[i] - st[i] for i in s) / 1e3
        span = (en[s[-1]] - st[s[0]]) / 1e3
        gaps = [(st[i] - en[i - 1]) / 1e3 for i in s[1:]]
        small = sum(g for g in gaps if g <= 10)
        big = [g for g in gaps if g > 10]
        short = sum(1 for i in s if (en[i] - st[i]) / 1e3 < 6)
        print(f"launches {len(s):5d} (<6us: {short:3d})  kernel {dur / 1e3:7.3f} ms  span "
              f"{span / 1e3:7.3f} ms  small gaps {small / 1e3:6.3f} ms  large gaps "
              f"{len(big):3d} = {sum(big) / 1e3:6.3f} ms")


if __name__ == "__main__":
    main()
