"""Timeline of one halo_msm_batch_dev call from a rocprofv3 kernel trace: per kernel name, start/end
relative to the first kernel (us), to see whether the fronts overlap the accumulations.
usage: python tools/trace_batch.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last batch: the final 60 kernels or so
acc = [i for i, r in enumerate(rows) if "k_acc<" in r["Kernel_Name"]]
first = acc[-8] - 12 if len(acc) >= 8 else 0
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:]:
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("halo::", "")[:40]
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r.get('Queue_Id', '?'):>3} {nm}")
