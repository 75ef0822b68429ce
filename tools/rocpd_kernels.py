#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 SQLite output (run_results.db):
count, median, min and total microseconds per kernel name."""
import collections
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    st = collections.defaultdict(list)
    for name, start, end in c.execute("select name, start, end from kernels"):
        st[name].append((end - start) / 1000.0)
    for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{len(v):5d} med {v[len(v) // 2]:9.1f} us  min {v[0]:9.1f}  total {sum(v):10.1f}  {k[:100]}")


if __name__ == "__main__":
    main(sys.argv[1])
