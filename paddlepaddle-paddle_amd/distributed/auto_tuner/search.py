"""Search algorithms of the auto tuner (reference: python/paddle/distributed/auto_tuner/search.py —
GridSearch, CustomizeSearch; plus a cost-model-ordered search of this framework)."""
from .prune import prune
from .utils import search_all, cfg_key
from .cost_model import estimate_step_time


class SearchAlgo:
    def __init__(self, tuner_cfg):
        self.tuner_cfg = tuner_cfg
        self.pruned = []  # (cfg, reason)

    def search_once(self, history_cfgs):
        raise NotImplementedError


class GridSearch(SearchAlgo):
    """Every candidate in a fixed order (memory-friendliest layouts last: larger mp / pp, smaller
    micro batch), skipping pruned ones against the history so far."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        self.all = self._order(search_all(tuner_cfg))
        self.idx = 0

    def _order(self, cfgs):
        return sorted(cfgs, key=lambda c: (c['mp_degree'] * c['pp_degree'], -c['micro_batch_size'],
                                           bool(c.get('use_recompute')), c['dp_degree']))

    def search_once(self, history_cfgs):
        seen = {cfg_key(h) for h in history_cfgs}
        while self.idx < len(self.all):
            cfg = dict(self.all[self.idx])
            self.idx += 1
            if cfg_key(cfg) in seen:
                continue
            reason = prune(self.tuner_cfg, cfg, history_cfgs)
            if reason:
                self.pruned.append((cfg, reason))
                continue
            return cfg
        return None


class CostModelSearch(GridSearch):
    """Grid candidates ordered by the analytic MI355X step-time model (cost_model.py): the
    predicted-fastest layouts run first, so a small ``task_limit`` still finds the winner."""

    def _order(self, cfgs):
        m = self.tuner_cfg['model_cfg']
        n = int(self.tuner_cfg.get('num_gpus', 8))
        gpn = int(self.tuner_cfg.get('gpus_per_node', 8))
        for c in cfgs:
            c['estimated_step_time'] = estimate_step_time(m, c, n, gpn) if c.get('acc_steps') else float('inf')
        return sorted(cfgs, key=lambda c: c['estimated_step_time'])


class CustomizeSearch(SearchAlgo):
    """The user's own list of configs (``tuner_cfg['configs']``), in order."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        self.cfgs = [dict(c) for c in tuner_cfg.get('configs', [])]
        self.idx = 0

    def search_once(self, history_cfgs):
        if self.idx >= len(self.cfgs):
            return None
        self.idx += 1
        return self.cfgs[self.idx - 1]
