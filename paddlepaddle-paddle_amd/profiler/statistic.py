"""Summary tables (reference: python/paddle/profiler/profiler_statistic.py — overview,
operator/UDF, kernel and memcpy views, sortable by SortedKeys)."""
from collections import defaultdict

_UNIT = {'s': 1e9, 'ms': 1e6, 'us': 1e3, 'ns': 1.0}


def _agg(events):
    d = defaultdict(lambda: [0, 0, 0, float('inf')])  # calls, total, max, min
    for e in events:
        dur = e['end'] - e['start']
        a = d[e['name']]
        a[0] += 1
        a[1] += dur
        a[2] = max(a[2], dur)
        a[3] = min(a[3], dur)
    return d


def _table(title, rows, unit, total):
    scale = _UNIT[unit]
    w = max([len(r[0]) for r in rows] + [20])
    w = min(w, 90)
    lines = [f"{'-' * (w + 70)}", f"{title}", f"{'-' * (w + 70)}",
             f"{'Name':<{w}}  {'Calls':>7}  {'Total(' + unit + ')':>12}  {'Avg':>10}  {'Max':>10}  {'Min':>10}  "
             f"{'Ratio(%)':>8}"]
    for name, (calls, tot, mx, mn) in rows:
        lines.append(f"{name[:w]:<{w}}  {calls:>7}  {tot / scale:>12.3f}  {tot / calls / scale:>10.3f}  "
                     f"{mx / scale:>10.3f}  {mn / scale:>10.3f}  {100.0 * tot / max(total, 1):>8.2f}")
    return '\n'.join(lines)


def build_summary(result, sorted_by, unit='ms', views=None):
    from .profiler import SortedKeys, SummaryView
    key = {SortedKeys.CPUTotal: 1, SortedKeys.GPUTotal: 1, SortedKeys.CPUAvg: 'avg', SortedKeys.GPUAvg: 'avg',
           SortedKeys.CPUMax: 2, SortedKeys.GPUMax: 2, SortedKeys.CPUMin: 3, SortedKeys.GPUMin: 3}[sorted_by]

    def order(d):
        items = list(d.items())
        if key == 'avg':
            return sorted(items, key=lambda kv: -kv[1][1] / kv[1][0])
        return sorted(items, key=lambda kv: (kv[1][key] if key == 3 else -kv[1][key]))

    views = set(views) if views is not None else None
    out = []
    steps = result.steps
    if views is None or SummaryView.OverView in views:
        if steps:
            tot = sum(t for _, t in steps)
            out.append(f"{'-' * 60}\nOverview: {len(steps)} steps, avg step {tot / len(steps) / _UNIT[unit]:.3f} {unit}")
    host = [e for e in result.host if e['type'] != 'ProfileStep']
    span = sum(t for _, t in steps) or 1
    if host and (views is None or SummaryView.OperatorView in views or SummaryView.UDFView in views):
        out.append(_table('Host ranges (RecordEvent / Optimization / Dataloader)', order(_agg(host)), unit, span))
    kern = [e for e in result.device if e['type'] == 'Kernel']
    if kern and (views is None or SummaryView.KernelView in views or SummaryView.DeviceView in views):
        ktot = sum(e['end'] - e['start'] for e in kern)
        out.append(_table('Device kernels', order(_agg(kern)), unit, ktot))
    mem = [e for e in result.device if e['type'] in ('Memcpy', 'Memset')]
    if mem and (views is None or SummaryView.MemoryManipulationView in views):
        mtot = sum(e['end'] - e['start'] for e in mem)
        out.append(_table('Memory copies / sets', order(_agg(mem)), unit, mtot))
    return '\n'.join(out)
