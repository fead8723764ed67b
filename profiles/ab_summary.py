"""Summarise a profiles/fit_ab.sh run: per variant, the wall time line and the top kernels."""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
i = 0
while os.path.exists(f'{d}/v{i}.env'):
    print('==', open(f'{d}/v{i}.env').read().strip())
    for line in open(f'{d}/v{i}.log'):
        if 'ms per' in line or 'M/s' in line:
            print('  ', line.strip())
    fs = glob.glob(f'{d}/v{i}/**/*kernel_stats.csv', recursive=True)
    if fs:
        for x in list(csv.DictReader(open(fs[0])))[:n]:
            print(f"   {x['Name'][:44]:44s} {x['Calls']:>6s} {float(x['AverageNs']) / 1000:8.2f} us")
    i += 1
