"""HBM traffic per launch of the bench's roofline kernel from scripts/pmc.sh's
FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 runs), with the gfx950
correction of MI355X_MICROARCH.md (FETCH_SIZE x2, WRITE_SIZE as reported; both
in KB), written as the profiles/<round>/pmc_traffic.json that bench.py reads.

  python scripts/pmc_traffic.py gpurun_out/pmc_bench3 profiles/r01/pmc_traffic.json [band GRID]

With `band` the kernel is the conv2 band reduction (band.hpp band_kernel; the
conv3 launch of the same kernel has another grid size: the dispatches are
grouped by grid size and the group with the larger mean FETCH_SIZE -- conv2 reads
a1, 2.5x conv3's a2 -- is taken; `band GRID` pins the grid size in threads).
"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = 'conv2 wgrad + K-FAC A-factor reduction GEMM (bf16x3 split-operand MFMA, f32-accurate)'
MATCH = 'symred6_kernel<acmi::CatRowsI<acmi::ConvRows<float, 20, 20, 32, 4, 4, 2>'
WORKLOAD = 'Breakout ACKTR 512 envs/GPU x 20 steps'
ALGO_INPUT_BYTES = 736624640  # a1 patches source + d2 read once (DESIGN.md Roofline)


BAND_KERNEL = ('conv2 band reduction: wgrad + K-FAC A factor over pixel-pair sub-tiles '
               '(f16x2 split-operand MFMA, f32-accurate)')
BAND_MATCH = 'band_kernel'
BAND = False
GRID = None


def per_dispatch(d, counter):
    vals = collections.defaultdict(float)
    grids = {}
    for f in glob.glob(os.path.join(d, '**', '*_counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row['Counter_Name'] == counter and MATCH in row['Kernel_Name']:
                    g = int(row.get('Grid_Size') or row.get('Grid_Size_X'))
                    if GRID is not None and g != GRID:
                        continue
                    key = (f, row['Dispatch_Id'])
                    vals[key] += float(row['Counter_Value'])
                    grids[key] = g
    if BAND and GRID is None and vals:
        by = collections.defaultdict(list)
        for k, v in vals.items():
            by[grids[k]].append(v)
        best = max(by, key=lambda g: sum(by[g]) / len(by[g]))
        return by[best]
    return list(vals.values())


def main(d, out):
    fetch = per_dispatch(d, 'FETCH_SIZE')
    write = per_dispatch(d, 'WRITE_SIZE')
    if not fetch or not write:
        raise SystemExit('no FETCH_SIZE/WRITE_SIZE samples for ' + MATCH)
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    res = {
        'kernel': KERNEL,
        'kernel_symbol_match': MATCH,
        'workload': WORKLOAD,
        'launches_sampled': min(len(fetch), len(write)),
        'fetch_size_kb_raw': f_kb,
        'write_size_kb_raw': w_kb,
        'correction': 'FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md '
                      'HBM section); WRITE_SIZE as reported',
        'hbm_bytes_per_launch': (2 * f_kb + w_kb) * 1024.0,
        'algorithmic_input_bytes': ALGO_INPUT_BYTES,
        'source': 'rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes, '
                  'bench.py --steps 3 --warmup 1 --no-cpu-baseline',
    }
    with open(out, 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    if len(sys.argv) > 3 and sys.argv[3] == 'band':
        KERNEL, MATCH, BAND = BAND_KERNEL, BAND_MATCH, True
        GRID = int(sys.argv[4]) if len(sys.argv) > 4 else None
    main(sys.argv[1], sys.argv[2])
