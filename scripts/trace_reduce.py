"""Keep the engine's kernels of a rocprofv3 kernel_trace.csv: name, start,
end and the queue / stream columns.  usage: trace_reduce.py <in.csv> <out.csv>"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "lkf::" in r["Kernel_Name"]]
keep = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"] + [k for k in rows[0] if "Queue" in k or "Stream" in k]
with open(sys.argv[2], "w") as f:
    w = csv.DictWriter(f, fieldnames=keep)
    w.writeheader()
    for r in rows:
        w.writerow({k: r[k] for k in keep})
print(len(rows), keep)
