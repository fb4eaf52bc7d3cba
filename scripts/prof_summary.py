"""Markdown table from a rocprofv3 --stats kernel_stats.csv.

  python scripts/prof_summary.py <kernel_stats.csv> <title> [iterations]
"""
import csv
import sys


def main(path, title, iters=None):
    rows = list(csv.DictReader(open(path)))
    print('# ' + title + '\n')
    print('| total ms | % | calls | avg us | per iter ms | kernel |')
    print('|---|---|---|---|---|---|')
    for r in rows:
        tot = float(r['TotalDurationNs']) / 1e6
        per = tot / iters if iters else float('nan')
        print('| {:.2f} | {:.1f} | {} | {:.1f} | {:.3f} | `{}` |'.format(
            tot, float(r['Percentage']), r['Calls'], float(r['AverageNs']) / 1e3, per, r['Name'][:150]))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
