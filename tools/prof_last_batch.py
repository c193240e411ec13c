"""Kernel time of the last timed call of a rocprofv3 kernel trace (sqlite
results.db): the kernels after the last-but-N occurrence of a marker kernel,
grouped by name.  python tools/prof_last_batch.py <results.db> [marker] [n]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_reduce_narrow"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    start = idx[-n] + 1
    agg = collections.OrderedDict()
    for name, t0, t1 in rows[start:]:
        a = agg.setdefault(name[:90], [0, 0.0])
        a[0] += 1
        a[1] += (t1 - t0) / 1e6
    for k, (cnt, ms) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{ms:9.3f} ms  n={cnt:4d}  {k}")
    print(f"kernel sum {sum(v[1] for v in agg.values()):.3f} ms, wall "
          f"{(rows[-1][2] - rows[start][1]) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
