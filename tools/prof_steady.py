"""Steady-state per-step kernel statistics from a rocprofv3 kernel_trace.csv.

Step boundaries are the dispatches of a kernel that runs once per training step (the fused
optimizer update); the last N steps (between the last N+1 markers) are aggregated, so
warmup-time work (library autotuning / MIOpen find, first-touch allocations) is excluded.

usage: prof_steady.py kernel_trace.csv MARKER_SUBSTRING N_STEPS [TOP]
"""
import csv
import sys

from prof_summary import cat


def main(path, marker, nsteps, top=30):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    # the first kernel name containing the substring is the marker (one bucket's update kernel)
    name = next((r['Kernel_Name'] for r in rows if marker in r['Kernel_Name']), None)
    marks = [i for i, r in enumerate(rows) if r['Kernel_Name'] == name]
    if len(marks) < nsteps + 1:
        raise SystemExit(f"only {len(marks)} '{marker}' dispatches, need {nsteps + 1}")
    lo, hi = marks[-(nsteps + 1)] + 1, marks[-1] + 1
    sel = rows[lo:hi]
    wall = (int(rows[hi - 1]['End_Timestamp']) - int(rows[lo]['Start_Timestamp'])) / 1e6 / nsteps
    per = {}
    for r in sel:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        t, c = per.get(r['Kernel_Name'], (0.0, 0))
        per[r['Kernel_Name']] = (t + d, c + 1)
    tot = sum(t for t, _ in per.values()) / nsteps
    print(f"steady state over the last {nsteps} steps: kernel time {tot:.2f} ms/step, "
          f"first-to-last dispatch span {wall:.2f} ms/step")
    groups = {}
    for n, (t, _) in per.items():
        groups[cat(n)] = groups.get(cat(n), 0.0) + t / nsteps
    for c, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"  {c:10s} {v:8.2f} ms  {100 * v / tot:5.1f}%")
    print("top kernels (ms/step, calls/step, avg us):")
    for n, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"  {t / nsteps:7.2f} {c / nsteps:6.1f} {1e3 * t / c:8.1f}  {n[:100]}")
    # GEMMs split by launch grid (one row per distinct shape)
    def grid(r):
        g = [r.get(k) for k in ('Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z') if r.get(k)]
        return 'x'.join(g) if g else r.get('Grid_Size', '?')
    shp = {}
    for r in sel:
        if 'gemm' not in r['Kernel_Name'] and 'Cijk' not in r['Kernel_Name']:
            continue
        k = (r['Kernel_Name'][:60], grid(r))
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        t, c = shp.get(k, (0.0, 0))
        shp[k] = (t + d, c + 1)
    if shp:
        print("GEMM kernels by launch grid (ms/step, calls/step, avg us, grid):")
        for (n, g), (t, c) in sorted(shp.items(), key=lambda kv: -kv[1][0]):
            print(f"  {t / nsteps:7.2f} {c / nsteps:6.1f} {1e3 * t / c:8.1f}  {g:>14s}  {n}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 30)
