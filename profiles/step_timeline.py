"""Print one step's kernel timeline from a rocprofv3 kernel trace CSV (gaps, durations).

usage: python profiles/step_timeline.py <run_kernel_trace.csv> [anchor kernel substring] [which: -2]
The step is the span between two consecutive launches of the anchor kernel (default k_expand).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else 'k_expand'
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if anchor in r['Kernel_Name']]
    a, b = idx[which], idx[which + 1]
    t0 = prev = int(rows[a]['Start_Timestamp'])
    busy = 0
    for r in rows[a:b]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} gap {(s - prev) / 1e3:7.1f} dur {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:80]}")
        prev = max(prev, e)
    span = int(rows[b]['Start_Timestamp']) - t0
    print(f'step span {span / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us')


if __name__ == '__main__':
    main()
