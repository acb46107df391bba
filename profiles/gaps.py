"""Idle gaps between kernels in a rocprofv3 kernel trace (diagnostic).

usage: python profiles/gaps.py <kernel_trace.csv> [window_s] [min_gap_us]
Looks at the last `window_s` seconds of the trace (e.g. a timed cycle) and reports the
busy time, the idle time in gaps >= min_gap_us and the largest gaps with their neighbours."""
import csv
import sys
from collections import Counter


def main():
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
            for r in csv.DictReader(open(sys.argv[1]))]
    rows.sort()
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 1e9
    mg = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    t_end = max(e for _, e, _ in rows)
    rows = [r for r in rows if r[0] >= t_end - win * 1e9]
    t0 = rows[0][0]
    busy, idle, gaps, cur = 0, 0, [], t0
    for s, e, n in rows:
        if s > cur:
            g = (s - cur) / 1e3
            if g >= mg:
                idle += s - cur
                gaps.append((g, prev, n))
        busy += e - s
        cur = max(cur, e)
        prev = n
    span = (cur - t0) / 1e9
    print(f"span {span:.3f} s, kernel time {busy / 1e9:.3f} s, idle in gaps >= {mg} us: {idle / 1e9:.3f} s, "
          f"{len(rows)} kernels")
    gaps.sort(reverse=True)
    for g, a, b in gaps[:15]:
        print(f"  {g:10.1f} us  after {a[:60]}  before {b[:60]}")
    c = Counter((a[:50], b[:50]) for _, a, b in gaps)
    print("most frequent gap sites:")
    for (a, b), k in c.most_common(8):
        print(f"  {k:6d}  {a} -> {b}")


if __name__ == "__main__":
    main()
