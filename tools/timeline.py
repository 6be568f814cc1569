# Step anatomy of the pipelined MSM bench from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv):
#   python3 tools/timeline.py <kernel_trace.csv> [k_acc launches to skip]
# For each k_acc launch after the skipped ones: the front kernels on its stream since the previous k_acc
# (start/end relative to the previous k_acc's end), k_acc's duration, and which tail kernels overlapped
# the front and k_acc.  Prints per-step rows and the averages.
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("halo::", "")
    return n[:40]


ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
               r.get("Queue_Id", r.get("Stream_Id", "?"))))
ks.sort()
acc = [k for k in ks if k[2].startswith("k_acc")]
steps = []
for i in range(max(1, skip), len(acc)):
    prev_end = acc[i - 1][1]
    a0, a1 = acc[i][0], acc[i][1]
    front = [k for k in ks if k[0] >= prev_end - 1000 and k[1] <= a0 + 1000 and k[2].startswith("k_rs")]
    f0 = min((k[0] for k in front), default=a0)
    f1 = max((k[1] for k in front), default=a0)
    tails = sorted({k[2] for k in ks if k[0] < a1 and k[1] > prev_end and not k[2].startswith(("k_rs", "k_acc"))})
    steps.append(dict(step=a1 - prev_end, gap_before_front=f0 - prev_end, front=f1 - f0, gap_front_acc=a0 - f1,
                      acc=a1 - a0, kernels=[(k[2], k[0] - prev_end, k[1] - k[0]) for k in front], tails=tails))
for s in steps:
    print("step %7.1f us: gap %5.1f front %6.1f gap %5.1f acc %6.1f | %s" % (
        s["step"] / 1e3, s["gap_before_front"] / 1e3, s["front"] / 1e3, s["gap_front_acc"] / 1e3, s["acc"] / 1e3,
        " ".join("%s@%.0f+%.0f" % (n.replace("k_rs_", ""), t0 / 1e3, d / 1e3) for n, t0, d in s["kernels"])))
if steps:
    m = len(steps)
    for key in ("step", "gap_before_front", "front", "gap_front_acc", "acc"):
        print("avg %-17s %7.1f us" % (key, sum(s[key] for s in steps) / m / 1e3))
    print("tail kernels overlapping the steps:", sorted({t for s in steps for t in s["tails"]}))
