"""Write the rocprofv3 `--stats` kernel summary (the *_kernel_stats.csv columns)
from a rocprofv3 results database (`<name>_results.db`, the default output
format of ROCm 7.2 when no --output-format is given).

usage: python scripts/db_kernel_stats.py <results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute('select name, count(*), sum(duration), avg(duration), min(duration), max(duration), '
                     'avg(duration * duration) from kernels group by name order by sum(duration) desc').fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs', 'StdDev'])
        for name, n, tot, avg, mn, mx, sq in rows:
            std = max(sq - avg * avg, 0.0) ** 0.5
            w.writerow([name, n, tot, f'{avg:.1f}', f'{100.0 * tot / total:.4f}', mn, mx, f'{std:.1f}'])
    print(f'{len(rows)} kernels -> {out}')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
