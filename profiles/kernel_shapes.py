"""Group a rocprofv3 kernel trace by (kernel, grid) and print the top shapes.

usage: python profiles/kernel_shapes.py <kernel_trace.csv> [top=30]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    agg = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = (row.get("Grid_Size_X", row.get("Grid_Size", "?")), row.get("Grid_Size_Y", ""),
                row.get("Grid_Size_Z", ""))
        dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
        a = agg[(name, grid)]
        a[0] += 1
        a[1] += dur
        total += dur
    print(f"total kernel time {total / 1e3:.1f} ms")
    byname = defaultdict(float)
    for (n, _), (c, t) in agg.items():
        byname[n] += t
    for n, t in sorted(byname.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {t / total * 100:5.1f}%  {t / 1e3:9.1f} ms  {n}")
    print("by shape:")
    for (n, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {t / total * 100:5.1f}%  n={c:5d}  avg {t / c:9.1f} us  grid={'x'.join(x for x in g if x)}  {n}")


if __name__ == "__main__":
    main()
