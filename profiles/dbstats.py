#!/usr/bin/env python3
"""Per-kernel time statistics from a rocprofv3 rocpd database (when --output-format csv was not given).
usage: python profiles/dbstats.py run_results.db [name-substring ...]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    pats = sys.argv[2:]
    rows = db.execute('select name, count(*), avg("end" - start), min("end" - start), max("end" - start) '
                      'from kernels group by name order by sum("end" - start) desc').fetchall()
    for name, c, avg, lo, hi in rows:
        if pats and not any(p in name for p in pats):
            continue
        print(f'  {name[:44]:44s} {c:5d} avg {avg / 1e3:8.1f} us  min {lo / 1e3:8.1f}  max {hi / 1e3:8.1f}')


if __name__ == '__main__':
    main()
