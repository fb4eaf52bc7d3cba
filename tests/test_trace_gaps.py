"""scripts/trace_gaps.py (the per-iteration launch / idle-gap table of a rocprofv3
kernel trace, committed with the small-config profiles) on a synthetic trace."""
import csv
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_trace_gaps_counts_busy_idle_and_launches(tmp_path):
    # three iterations delimited by returns_kernel; per iteration: returns 10 us,
    # a gap of 5 us, band 30 us overlapping a 10-us fill, a gap of 25 us
    rows = []
    t = 1000000
    for it in range(3):
        rows.append(('acmi::returns_kernel(float const*)', t, t + 10000))
        rows.append(('acmi::band_kernel(acmi::BandArgs)', t + 15000, t + 45000))
        rows.append(('__amd_rocclr_fillBufferAligned', t + 20000, t + 30000))
        t += 70000
    rows.append(('acmi::returns_kernel(float const*)', t, t + 10000))
    path = tmp_path / 'kernel_trace.csv'
    with open(path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
        for r in rows:
            w.writerow(r)
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'trace_gaps.py'), str(path)],
                         capture_output=True, text=True, check=True).stdout
    assert '3 iterations' in out
    assert '| wall span (first kernel start to next iteration) | 0.070 ms |' in out
    assert '| GPU busy (union of kernel intervals) | 0.040 ms (57.1 %) |' in out
    assert '| kernel launches | 3.0 |' in out
    assert '| gaps > 20 us: count / total per iteration | 1.0 / 0.025 ms |' in out
    # skipping the first iteration (warm-up) leaves two
    out2 = subprocess.run([sys.executable, os.path.join(ROOT, 'scripts', 'trace_gaps.py'), str(path),
                           'returns_kernel', '1'], capture_output=True, text=True, check=True).stdout
    assert '2 iterations' in out2
