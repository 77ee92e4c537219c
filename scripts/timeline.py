"""Print one step's kernel timeline from a rocprofv3 kernel_trace.csv:
start/end (us, relative to the step's first kernel) per lkf kernel dispatch.
usage: python3 scripts/timeline.py <kernel_trace.csv> [step_index]
A step is delimited by k_ing_init (ingest step) or k_batch_init (forward step)."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "lkf::" not in n:
        continue
    short = n.split("(")[0].replace("void ", "").replace("lkf::", "").replace("(anonymous namespace)::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
rows.sort()
mark = "k_ing_init" if any(s == "k_ing_init" for _, _, s in rows) else "k_batch_init"
starts = [i for i, (_, _, s) in enumerate(rows) if s == mark]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
a, b = starts[k], starts[k + 2] if k + 2 < len(starts) else len(rows)
t0 = rows[a][0]
period = (rows[starts[k + 1]][0] - t0) / 1000 if k + 1 < len(starts) else 0
print("step %d: period to the next %s: %.1f us" % (k, mark, period))
for s, e, n in rows[a:b]:
    print("%9.1f %9.1f %8.1f  %s" % ((s - t0) / 1000, (e - t0) / 1000, (e - s) / 1000, n))
