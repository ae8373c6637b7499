"""AutoTuner (reference: python/paddle/distributed/auto_tuner/tuner.py): hands out candidate
hybrid-parallel configs, records their results, reports the best.  ``run`` drives trials through
a caller-supplied function (the launcher's ``--auto_tuner_json`` mode starts the real jobs)."""
import json
import os

from .recorder import HistoryRecorder
from .utils import default_candidates, cfg_key


class AutoTuner:
    def __init__(self, tuner_cfg):
        if isinstance(tuner_cfg, str):
            with open(tuner_cfg) as f:
                tuner_cfg = json.load(f)
        tuner_cfg = dict(tuner_cfg)
        tuner_cfg.setdefault('num_gpus', int(tuner_cfg.get('nodes', 1)) * int(tuner_cfg.get('gpus_per_node', 8)))
        self.cur_task_id = 1
        self.task_limit = int(tuner_cfg.get('task_limit', 100))
        algo = (tuner_cfg.get('search_algo') or {'name': 'grid'})['name']
        tuner_cfg['candidates'] = default_candidates(tuner_cfg)
        from . import search
        if algo == 'grid':
            self.algo = search.GridSearch(tuner_cfg)
        elif algo in ('cost_model', 'dp_estimation'):
            self.algo = search.CostModelSearch(tuner_cfg)
        elif algo == 'customize':
            self.algo = search.CustomizeSearch(tuner_cfg)
        else:
            raise NotImplementedError(f"search_algo {algo!r}")
        self.tuner_cfg = tuner_cfg
        self.history_cfgs = []
        self.resume_cfgs = []
        self.recorder = HistoryRecorder(tuner_cfg)

    def search_once(self):
        """The next config to run (None when the space or ``task_limit`` is exhausted)."""
        if self.cur_task_id > self.task_limit:
            return None
        cfg = self.algo.search_once(self.history_cfgs)
        if cfg is not None:
            cfg['job_id'] = self.cur_task_id
        self.cur_task_id += 1
        return cfg

    def add_cfg(self, cfg):
        """Record a finished trial (cfg with the metric, ``time`` = -1 on failure, ``oom``)."""
        self.history_cfgs.append(cfg)
        self.recorder.add_cfg(**cfg)

    def get_best(self):
        best, err = self.recorder.get_best()
        return None if err else best

    def resume_form_history(self, history_csv_path='./history.csv'):
        if os.path.exists(history_csv_path):
            self.resume_cfgs = HistoryRecorder(self.tuner_cfg).load_history(history_csv_path)

    def get_cfg_from_resume(self, cur_cfg):
        k = cfg_key(cur_cfg)
        for c in self.resume_cfgs:
            if cfg_key(c) == k:
                return c
        return None

    def run(self, trial_fn, history_csv_path=None):
        """Run trials until the search ends: ``trial_fn(cfg)`` returns the metric value (None on
        failure) or a dict of fields to record (metric, ``oom``).  Returns the best config."""
        metric = self.recorder.metric
        while True:
            cfg = self.search_once()
            if cfg is None:
                break
            prev = self.get_cfg_from_resume(cfg)
            res = prev if prev is not None else trial_fn(dict(cfg))
            rec = dict(cfg)
            if isinstance(res, dict):
                rec.update(res)
            else:
                rec[metric] = -1 if res is None else res
            rec.setdefault('time', rec.get(metric, -1))
            self.add_cfg(rec)
            if history_csv_path:
                self.recorder.store_history(history_csv_path)
        return self.get_best()
