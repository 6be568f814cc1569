"""Prints the kernel sequence of a rocprofv3 kernel_trace.csv between two timestamps (relative ms)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
t0 = min(int(r['Start_Timestamp']) for r in rows)
lo, hi = float(sys.argv[2]), float(sys.argv[3])
for r in sorted(rows, key=lambda r: int(r['Start_Timestamp'])):
    s = (int(r['Start_Timestamp']) - t0) / 1e6
    e = (int(r['End_Timestamp']) - t0) / 1e6
    if lo <= s <= hi:
        print(f"{s:10.3f} {e - s:8.3f} ms  q{r.get('Queue_Id', '?')}  {r['Kernel_Name'][:80]}")
