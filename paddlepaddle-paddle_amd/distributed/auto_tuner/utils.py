"""Candidate generation for the auto tuner (reference: python/paddle/distributed/auto_tuner/utils.py
default_candidates / search_all)."""
import itertools

_DIMS = ('dp_degree', 'mp_degree', 'pp_degree', 'vpp_degree', 'sharding_degree', 'sharding_stage',
         'micro_batch_size', 'use_recompute', 'recompute_granularity')


def divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def _num_gpus(tuner_cfg):
    return int(tuner_cfg.get('num_gpus', int(tuner_cfg.get('nodes', 1)) * int(tuner_cfg.get('gpus_per_node', 8))))


def default_candidates(tuner_cfg):
    """Value lists per search dimension: a list in the config is taken as is, "auto" (or absent)
    expands to every value that can be valid for the machine / model."""
    n = _num_gpus(tuner_cfg)
    m = tuner_cfg.get('model_cfg', {})
    gbs = int(m.get('global_batch_size', 8))
    auto = {
        'dp_degree': divisors(n),
        'mp_degree': [d for d in divisors(n) if d <= int(tuner_cfg.get('gpus_per_node', 8))],
        'pp_degree': divisors(n),
        'vpp_degree': [1, 2],
        'sharding_degree': divisors(n),
        'sharding_stage': [1, 2, 3],
        'micro_batch_size': divisors(gbs),
        'use_recompute': [False, True],
        'recompute_granularity': ['full', 'full_attn', 'core_attn'],
    }
    out = {}
    for k in _DIMS:
        v = tuner_cfg.get(k, 'auto')
        out[k] = auto[k] if v in ('auto', None) else (list(v) if isinstance(v, (list, tuple)) else [v])
    return out


def search_all(tuner_cfg):
    """Every combination of the candidates that multiplies out to the GPU count (the rest of the
    pruning is prune.py's), with acc_steps filled in."""
    cand = tuner_cfg.get('candidates') or default_candidates(tuner_cfg)
    n = _num_gpus(tuner_cfg)
    gbs = int(tuner_cfg.get('model_cfg', {}).get('global_batch_size', 8))
    out = []
    for combo in itertools.product(*[cand[k] for k in _DIMS]):
        cfg = dict(zip(_DIMS, combo))
        if cfg['dp_degree'] * cfg['mp_degree'] * cfg['pp_degree'] * cfg['sharding_degree'] != n:
            continue
        if not cfg['use_recompute'] and cfg['recompute_granularity'] != cand['recompute_granularity'][0]:
            continue  # granularity is meaningless without recompute: keep one representative
        if not cfg['use_recompute']:
            cfg['recompute_granularity'] = None
        if cfg['sharding_degree'] == 1 and cfg['sharding_stage'] != cand['sharding_stage'][0]:
            continue
        if cfg['sharding_degree'] == 1:
            cfg['sharding_stage'] = None
        rep = cfg['dp_degree'] * cfg['sharding_degree']
        if gbs % rep or (gbs // rep) % cfg['micro_batch_size']:
            cfg['acc_steps'] = None
        else:
            cfg['acc_steps'] = gbs // rep // cfg['micro_batch_size']
        cfg['num_gpus'] = n
        cfg['global_batch_size'] = gbs
        out.append(cfg)
    return out


def cfg_key(cfg):
    return tuple((k, cfg.get(k)) for k in _DIMS)
