"""Trial history of the auto tuner (reference: python/paddle/distributed/auto_tuner/recorder.py)."""
import csv


class HistoryRecorder:
    def __init__(self, tuner_cfg=None):
        self.tuner_cfg = tuner_cfg or {}
        self.history = []
        m = self.tuner_cfg.get('metric_cfg', {})
        self.metric = m.get('name', 'time')
        self.direction = m.get('OptimizationDirection', 'Minimize' if self.metric == 'time' else 'Maximize')

    def add_cfg(self, **kwargs):
        self.history.append(dict(kwargs))

    def sort_metric(self):
        """Successful trials best first (failed / OOM trials last)."""
        ok = [h for h in self.history if h.get(self.metric) not in (None, -1) and not h.get('oom')]
        bad = [h for h in self.history if h not in ok]
        ok.sort(key=lambda h: float(h[self.metric]), reverse=self.direction.lower().startswith('max'))
        return ok + bad

    def get_best(self):
        s = self.sort_metric()
        if not s or s[0].get(self.metric) in (None, -1) or s[0].get('oom'):
            return None, True
        return s[0], False

    def store_history(self, path='./history.csv'):
        rows = self.sort_metric()
        keys = []
        for r in rows:
            for k in r:
                if k not in keys:
                    keys.append(k)
        with open(path, 'w', newline='') as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            for r in rows:
                w.writerow(r)

    def load_history(self, path='./history.csv'):
        with open(path) as f:
            rows = list(csv.DictReader(f))
        out = []
        for r in rows:
            d = {}
            for k, v in r.items():
                if v in ('', 'None'):
                    d[k] = None
                elif v in ('True', 'False'):
                    d[k] = v == 'True'
                else:
                    try:
                        d[k] = int(v)
                    except ValueError:
                        try:
                            d[k] = float(v)
                        except ValueError:
                            d[k] = v
            out.append(d)
        self.history = out
        return out
