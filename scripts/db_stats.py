"""Kernel statistics (calls, average / total µs) from a rocprofv3 sqlite
result (run_results.db), as the --stats CSV would list them."""
import collections
import sqlite3
import sys


def main(path, top=25):
    c = sqlite3.connect(path)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    agg = collections.defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        agg[names.get(kid, str(kid))].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print("Name,Calls,AverageNs,TotalNs,Percentage")
    for n, v in rows[:top]:
        print('"%s",%d,%.1f,%d,%.2f' % (n.split("(")[0], len(v), sum(v) / len(v), sum(v), 100.0 * sum(v) / tot))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
