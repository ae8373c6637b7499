"""Summarise a rocprofv3 kernel_stats.csv: per-kernel ms/step, grouped into categories."""
import csv
import sys


def cat(name):
    n = name.lower()
    if 'cijk' in n or 'gemm' in n:
        return 'gemm'
    if '2fa' in n or 'flash' in n:
        return 'attention'
    if 'adamw' in n or 'sumsq' in n:
        return 'optimizer'
    if 'conv' in n or 'miopen' in n or 'igemm' in n or 'xdlops' in n:
        return 'conv'
    if ('norm' in n or 'colsum' in n or 'act' in n or 'dropout' in n or 'xent' in n or 'embedding' in n
            or 'bn::' in n or '2bn' in n or 'momentum' in n):
        return 'fused-hip'
    return 'other'


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows) / 1e6 / steps
    groups = {}
    for r in rows:
        c = cat(r['Name'])
        groups[c] = groups.get(c, 0.0) + float(r['TotalDurationNs']) / 1e6 / steps
    print(f"total kernel time per step: {tot:.2f} ms")
    for c, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"  {c:10s} {v:8.2f} ms  {100 * v / tot:5.1f}%")
    print("top kernels (ms/step, calls/step, avg us):")
    for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
        print(f"  {float(r['TotalDurationNs']) / 1e6 / steps:7.2f} {int(r['Calls']) / steps:6.1f} "
              f"{float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]))
