"""Launch count, GPU-busy time and idle gaps per training iteration from a
rocprofv3 --kernel-trace CSV (kernel_trace.csv).

Iterations are delimited by a kernel that runs once per update (default
returns_kernel, the n-step target scan): the window from its first to its last
launch holds (count - 1) whole iterations.  Busy = the union of kernel
intervals; idle = window - busy (host launch latency, synchronisation,
dependency bubbles between back-to-back launches).

  python scripts/trace_gaps.py <kernel_trace.csv> [marker-substring] [skip] > gaps.md

skip: leading marker launches to drop (the warm-up iterations, whose first-use
plan builds and allocations would dominate the gaps).
"""
import csv
import sys


def main(path, marker='returns_kernel', skip=0):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        raise SystemExit('empty trace')
    keys = rows[0].keys()
    kname = next(k for k in keys if k.lower() in ('kernel_name', 'kernelname', 'name'))
    kbeg = next(k for k in keys if 'start' in k.lower())
    kend = next(k for k in keys if 'end' in k.lower())
    ev = sorted((int(r[kbeg]), int(r[kend]), r[kname]) for r in rows)
    marks = [b for b, e, n in ev if marker in n][int(skip):]
    if len(marks) < 2:
        raise SystemExit('marker {!r} seen {} times'.format(marker, len(marks)))
    w0, w1 = marks[0], marks[-1]
    iters = len(marks) - 1
    win = [(b, e, n) for b, e, n in ev if w0 <= b < w1]
    busy, cur_b, cur_e = 0, None, None
    gaps = []
    where = {}  # (kernel before, kernel after) -> idle ns
    short = lambda n: n.split('(')[0].split('<')[0].replace('void ', '').replace('acmi::', '')[:40]
    prev = None
    for b, e, n in win:
        if cur_e is None:
            cur_b, cur_e = b, e
        elif b > cur_e:
            busy += cur_e - cur_b
            gaps.append(b - cur_e)
            key = (short(prev), short(n))
            where[key] = where.get(key, 0) + (b - cur_e)
            cur_b, cur_e = b, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    busy += min(cur_e, w1) - cur_b
    if w1 > cur_e:  # the idle time before the next iteration's first kernel
        gaps.append(w1 - cur_e)
    span = w1 - w0
    per = lambda x: x / iters / 1e3
    print('# Kernel-trace timeline: {} iterations (window {} .. {} by `{}`)\n'.format(iters, w0, w1, marker))
    print('| per iteration | value |')
    print('|---|---|')
    print('| wall span (first kernel start to next iteration) | {:.3f} ms |'.format(per(span) / 1e3))
    print('| GPU busy (union of kernel intervals) | {:.3f} ms ({:.1f} %) |'.format(per(busy) / 1e3,
                                                                             100.0 * busy / span))
    print('| idle gaps | {:.3f} ms |'.format(per(span - busy) / 1e3))
    print('| kernel launches | {:.1f} |'.format(len(win) / iters))
    print('| gaps between kernels | {:.1f} |'.format(len(gaps) / iters))
    if gaps:
        gs = sorted(gaps)
        q = lambda f: gs[min(len(gs) - 1, int(f * len(gs)))] / 1e3
        print('| gap median / p90 / max | {:.1f} / {:.1f} / {:.1f} us |'.format(q(0.5), q(0.9), gs[-1] / 1e3))
        big = [g for g in gaps if g > 20000]
        print('| gaps > 20 us: count / total per iteration | {:.1f} / {:.3f} ms |'.format(
            len(big) / iters, sum(big) / iters / 1e6))
    print('\n| idle before | after | us / iter |')
    print('|---|---|---|')
    for k in sorted(where, key=lambda x: -where[x])[:12]:
        print('| `{}` | `{}` | {:.1f} |'.format(k[0], k[1], per(where[k])))
    tot = {}
    cnt = {}
    for b, e, n in win:
        k = n.split('(')[0][:90]
        tot[k] = tot.get(k, 0) + (e - b)
        cnt[k] = cnt.get(k, 0) + 1
    print('\n| kernel | launches / iter | us / iter | us / launch |')
    print('|---|---|---|---|')
    for k in sorted(tot, key=lambda x: -tot[x])[:25]:
        print('| `{}` | {:.1f} | {:.1f} | {:.1f} |'.format(k, cnt[k] / iters, per(tot[k]), tot[k] / cnt[k] / 1e3))


if __name__ == '__main__':
    main(*sys.argv[1:])
