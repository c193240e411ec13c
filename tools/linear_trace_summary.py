"""Median duration per teacher-Linear launch shape from a rocprofv3 kernel
trace (csv): python tools/linear_trace_summary.py <trace.csv> <label>"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "teacher_linear" in r["Kernel_Name"]:
        agg[r["Grid_Size_X"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(json.dumps(dict(label=sys.argv[2], median_us={k: sorted(v)[len(v) // 2]
                                                      for k, v in agg.items()},
                      launches={k: len(v) for k, v in agg.items()})))
