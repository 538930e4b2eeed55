"""Print the top kernels of a rocprofv3 kernel_stats.csv: name, calls, avg ms, total ms."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    rows = list(csv.DictReader(open(path)))
    for r in rows[:16]:
        print(f"  {r['Name'][:78]:80s} {r['Calls']:>5s} {float(r['AverageNs'])/1e6:8.3f} {float(r['TotalDurationNs'])/1e6:9.2f}")
