"""Mean duration per (kernel, grid) from a rocprofv3 kernel trace (csv), the
heaviest first: python tools/kernel_trace_summary.py <kernel_trace.csv> [top]

Used for the per-layer FedDF teacher profiles under profiles/ (the kernel's
own launches only; the torch kernels of the vmap'd segments show up too)."""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    agg = collections.defaultdict(list)
    for r in rows:
        key = (short(r["Kernel_Name"]),
               "(%s,%s,%s)" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]),
               r["Workgroup_Size_X"])
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    for (name, grid, wg), us in tot[:top]:
        print("%10.1f us  n=%4d  total %9.1f us  %-70s grid=%s wg=%s"
              % (sum(us) / len(us), len(us), sum(us), name, grid, wg))


if __name__ == "__main__":
    main()
