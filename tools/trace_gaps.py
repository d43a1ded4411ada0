"""Per-kernel average duration and the average idle gap before each kernel
(previous dispatch end -> this start) from a rocprofv3 --kernel-trace CSV.
usage: python tools/trace_gaps.py run_kernel_trace.csv [name_substring ...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
want = sys.argv[2:]
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
prev_end = None
for r in rows:
    n, s, e = r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not want or any(w in n for w in want):
        dur[n] += e - s
        cnt[n] += 1
        if prev_end is not None:
            gap[n] += max(0, s - prev_end)
    prev_end = e
for n in sorted(cnt, key=lambda k: -dur[k]):
    print(f"{n[:40]:40s} calls {cnt[n]:6d}  avg {dur[n] / cnt[n] / 1e3:8.2f} us  gap before {gap[n] / cnt[n] / 1e3:7.2f} us")
