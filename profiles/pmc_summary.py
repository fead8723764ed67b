"""Aggregate rocprofv3 --pmc counter CSVs per kernel name.
usage: python profiles/pmc_summary.py <dir-with-pass-subdirs> [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pats = sys.argv[2:]
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(root, '*', '*counter_collection.csv')) + glob.glob(
            os.path.join(root, '*', '*', '*counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            name = r.get('Kernel_Name', r.get('Kernel-Name', ''))
            name = name.split('(')[0]
            if pats and not any(p in name for p in pats):
                continue
            c = r.get('Counter_Name', r.get('Counter-Name'))
            v = float(r.get('Counter_Value', r.get('Counter-Value', 0)))
            agg[name][c] += v
            cnt[name][c] += 1
    for name, cs in sorted(agg.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f'   {c:28s} {v:16.0f}  (per dispatch {v / max(1, cnt[name][c]):14.1f})')


if __name__ == '__main__':
    main()
