"""One training iteration of a rocprofv3 kernel trace as a per-queue timeline
(start offset, duration, gap to the previous kernel end, queue): under the
side-stream G chain the stats summary's per-kernel durations include the time a
kernel's blocks wait for CU slots held by the other stream's kernels, so the
critical path is read here.  The rollout's per-step kernels are folded into one
line per kernel name.

  python scripts/iter_timeline.py <kernel_trace.csv> [iteration index] > timeline.md
  python scripts/iter_timeline.py <kernel_trace.csv> band   (the band launches by shape)
"""
import collections
import csv
import re
import sys


def main(path, it=4):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    marks = [i for i, r in enumerate(rows) if 'returns_kernel' in r['Kernel_Name']]
    a, b = marks[it], marks[it + 1]
    t0 = int(rows[a]['Start_Timestamp'])
    print('# One iteration (returns_kernel #%d to #%d) of %s\n' % (it, it + 1, path.split('/')[-1]))
    print('| start us | dur us | queue | kernel |')
    print('|---|---|---|---|')
    folded = collections.OrderedDict()
    for r in rows[a:b]:
        n = re.sub(r'\(.*', '', r['Kernel_Name']).replace('acmi::', '').replace('void ', '')[:90]
        s = (int(r['Start_Timestamp']) - t0) / 1e3
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        if 'rollout_tail' in n or 'fc4_roll' in n:
            f = folded.setdefault(n, [s, 0.0, 0])
            f[1] += d
            f[2] += 1
            continue
        print('| %.1f | %.1f | %s | `%s` |' % (s, d, r['Queue_Id'], n))
    end = (int(rows[b]['Start_Timestamp']) - t0) / 1e3
    for n, (s, tot, cnt) in folded.items():
        print('| %.1f | %.1f (%d launches, %.1f each) | rollout | `%s` |' % (s, tot, cnt, tot / cnt, n))
    print('\niteration span: %.1f us' % end)


def band_by_grid(path, warm=2):
    """The band reductions by launch shape (conv2 and conv3 share `band_kernel`, the stats
    summary averages them together): mean duration over all launches and after the
    first `warm` (the bench's warm-up iterations)."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    d = collections.OrderedDict()
    for r in rows:
        if 'band_kernel' in r['Kernel_Name']:
            d.setdefault(r['Grid_Size_X'], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    print('| band launch (grid threads) | launches | mean us | mean us after %d |' % warm)
    print('|---|---|---|---|')
    for g, v in d.items():
        print('| %s | %d | %.1f | %.1f |' % (g, len(v), sum(v) / len(v), sum(v[warm:]) / max(1, len(v[warm:]))))


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[2] == 'band':
        band_by_grid(sys.argv[1])
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
