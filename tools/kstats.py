"""Summarise a rocprofv3 kernel_stats.csv: name, calls, average us, share."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for x in list(csv.DictReader(open(path)))[:int(__import__("os").environ.get("TOP", "20"))]:
        print(f"{x['Name'][:96]:96s} {x['Calls']:>6} {float(x['AverageNs'])/1e3:8.1f}us {float(x['Percentage']):5.1f}%")
