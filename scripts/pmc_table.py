"""Summarise scripts/pmc.sh output: per kernel (short name), mean of each
counter over its dispatches.   python scripts/pmc_table.py gpurun_out/pmc_bwd"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r'gemm_kernel<([^>]*?)(,\s*acmi::([A-Za-z]+)<[^,]*?(\w+)?)', name)
    name = re.sub(r'\(.*', '', name)
    name = name.replace('acmi::', '').replace('void ', '')
    return name[:150]


def main(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, '*', '*_counter_collection.csv')):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row['Kernel_Name'])
                g = row.get('Grid_Size') or row.get('Grid_Size_X')
                if g:  # one kernel at several shapes (the band reductions of conv2 / conv3)
                    k = '{} [grid {}]'.format(k, g)
                vals[k][row['Counter_Name']].append((row['Dispatch_Id'], float(row['Counter_Value'])))
    for k, cs in sorted(vals.items()):
        print(k)
        for c, v in sorted(cs.items()):
            per = collections.defaultdict(float)
            for disp, x in v:
                per[disp] += x
            xs = list(per.values())
            print('   {:28s} {:16.4g}  (n={})'.format(c, sum(xs) / len(xs), len(xs)))


if __name__ == '__main__':
    main(sys.argv[1])
