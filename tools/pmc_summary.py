"""Summarise rocprofv3 --pmc CSV output: per kernel (last dispatch), counters + derived clock /
MFMA utilisation.  usage: pmc_summary.py <dir with v*/ subdirs or counter_collection csvs>"""
import csv
import glob
import os
import sys


def main(root):
    files = sorted(glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True))
    for f in files:
        rows = list(csv.DictReader(open(f)))
        per = {}
        for r in rows:
            key = (r['Dispatch_Id'], r['Kernel_Name'])
            per.setdefault(key, {})[r['Counter_Name']] = float(r['Counter_Value'])
            per[key]['_dur'] = None
        # last dispatch of each distinct kernel name
        last = {}
        for (d, k), c in per.items():
            if k not in last or int(d) > int(last[k][0]):
                last[k] = (d, c)
        kt = glob.glob(os.path.join(os.path.dirname(f), '*kernel_trace.csv'))
        dur = {}
        if kt:
            for r in csv.DictReader(open(kt[0])):
                dur[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        print('==', os.path.relpath(f, root))
        for k, (d, c) in sorted(last.items(), key=lambda x: x[0]):
            us = dur.get(d)
            print(f"  {k[:110]}")
            line = '   '
            for n in sorted(c):
                if n.startswith('_'):
                    continue
                line += f" {n}={c[n]:.4g}"
            print(line)
            wc = c.get('SQ_WAVE_CYCLES')
            if wc:
                print(f"    wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.1%} wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.1%}"
                      f" active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.1%}")
            if us and c.get('GRBM_GUI_ACTIVE'):
                clk = c['GRBM_GUI_ACTIVE'] / 8 / (us * 1e-6) / 1e9
                mf = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0)
                # MFMA busy cycles summed over SIMDs: utilisation = busy / (1024 SIMDs x active cycles)
                util = mf / (1024 * c['GRBM_GUI_ACTIVE'] / 8) if mf else 0
                print(f"    {us:.1f} us, effective clock {clk:.2f} GHz, MFMA pipe util {util:.1%}")


if __name__ == '__main__':
    main(sys.argv[1])
