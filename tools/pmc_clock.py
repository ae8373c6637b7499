"""Per-dispatch PMC summary with the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall) and
MFMA-pipe occupancy (SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES-based SIMD cycles)), from a
rocprofv3 --pmc counter_collection.csv.  Usage: pmc_clock.py <csv> [name-filter]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if filt not in r['Kernel_Name']:
            continue
        d = per.setdefault(r['Dispatch_Id'], {'name': r['Kernel_Name'], 't': (int(r['End_Timestamp']) - int(r['Start_Timestamp']))})
        d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    agg = collections.OrderedDict()
    for d in per.values():
        a = agg.setdefault(d['name'][:70], collections.defaultdict(float))
        for k, v in d.items():
            if k != 'name':
                a[k] += v
        a['n'] += 1
    for name, a in agg.items():
        t = a['t'] / a['n'] * 1e-9
        clk = a.get('GRBM_GUI_ACTIVE', 0) / a['n'] / 8 / t / 1e9 if t else 0
        wc = a.get('SQ_WAVE_CYCLES', 0)
        print(f"{name}\n   dispatches {int(a['n'])}  avg {t*1e6:8.1f} us  effective clock {clk:.2f} GHz")
        for k in sorted(x for x in a if x not in ('t', 'n')):
            if k in a:
                extra = f"  ({a[k] / wc * 100:5.1f} % of wave cycles)" if k.startswith('SQ_WAIT') and wc else ''
                print(f"   {k:26s} {a[k] / a['n']:16.0f}{extra}")
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in a and 'GRBM_GUI_ACTIVE' in a:
            # MFMA pipes: 256 CUs x 4 SIMDs; busy cycles are summed over SIMDs
            simd_cycles = a['GRBM_GUI_ACTIVE'] / 8 * 256 * 4
            print(f"   MFMA pipe busy {a['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles * 100:5.1f} % of SIMD cycles")
        if 'SQ_LDS_IDX_ACTIVE' in a and 'GRBM_GUI_ACTIVE' in a:
            # LDS-array cycles summed over CUs (one LDS per CU): share of the CU cycles the array is busy
            cu_cycles = a['GRBM_GUI_ACTIVE'] / 8 * 256
            print(f"   LDS array busy {a['SQ_LDS_IDX_ACTIVE'] / cu_cycles * 100:5.1f} % of CU cycles (SQ_LDS_IDX_ACTIVE)")
        if 'SQ_INSTS_VALU' in a and 'SQ_INSTS_MFMA' in a and a['SQ_INSTS_MFMA']:
            print(f"   VALU : MFMA instructions {a['SQ_INSTS_VALU'] / a['SQ_INSTS_MFMA']:.2f}")


if __name__ == '__main__':
    main()
