"""Group a rocprofv3 kernel_trace.csv by (kernel, grid): calls and mean device time (us)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else '')
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
    acc = defaultdict(list)
    order = []
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if filt and filt not in name:
            continue
        key = (name[:70], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Grid_Size_Y', ''))
        if key not in acc:
            order.append(key)
        acc[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for k in order:
        v = acc[k]
        v2 = sorted(v)[len(v) // 4:] or v  # drop the fastest quarter? keep median-ish: mean of upper 3/4
        print(f'{len(v):4d} calls  mean {sum(v) / len(v):8.2f} us  median {sorted(v)[len(v) // 2]:8.2f} us  '
              f'grid {k[1]}x{k[2]}  {k[0]}')


if __name__ == '__main__':
    main()
