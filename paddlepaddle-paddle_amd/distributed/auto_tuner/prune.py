"""Prune rules of the auto tuner (reference: python/paddle/distributed/auto_tuner/prune.py —
prune_by_mp / pp / vpp / mbs / sharding / recompute / num_gpus / memory_estimation and their
history forms).  A rule returns a reason string when the candidate is invalid, else None."""
from .memory_cost_model import estimate_memory_gb, model_dims

_RULES = []
_HISTORY_RULES = []


def register_prune(fn):
    _RULES.append(fn)
    return fn


def register_prune_history(fn):
    _HISTORY_RULES.append(fn)
    return fn


@register_prune
def prune_by_mp(tuner_cfg, cfg):
    d = model_dims(tuner_cfg['model_cfg'])
    mp = cfg['mp_degree']
    if d['a'] % mp or d['h'] % mp or d['f'] % mp or d['V'] % mp:
        return f"mp {mp} does not divide heads / hidden / ffn / vocab"
    if mp > int(tuner_cfg.get('gpus_per_node', 8)):
        return "tensor parallelism across nodes"
    return None


@register_prune
def prune_by_pp(tuner_cfg, cfg):
    L = model_dims(tuner_cfg['model_cfg'])['L']
    pp, vpp = cfg['pp_degree'], cfg.get('vpp_degree') or 1
    if L % (pp * vpp):
        return f"pp {pp} x vpp {vpp} does not divide {L} layers"
    if vpp > 1 and pp == 1:
        return "virtual stages without pipeline parallelism"
    acc = cfg.get('acc_steps')
    if pp > 1 and acc is not None and acc < pp:
        return f"accumulate steps {acc} < pp {pp}"
    if vpp > 1 and acc is not None and acc % pp:
        return "interleaved pipeline needs acc_steps % pp == 0"
    return None


@register_prune
def prune_by_mbs(tuner_cfg, cfg):
    if cfg.get('acc_steps') is None:
        return "micro batch does not divide the local batch"
    return None


@register_prune
def prune_by_sharding(tuner_cfg, cfg):
    if cfg['sharding_degree'] > 1 and cfg.get('sharding_stage') not in (1, 2, 3):
        return "sharding stage must be 1, 2 or 3"
    return None


@register_prune
def prune_by_num_gpus(tuner_cfg, cfg):
    n = cfg['dp_degree'] * cfg['mp_degree'] * cfg['pp_degree'] * cfg['sharding_degree']
    if n != cfg['num_gpus']:
        return f"degrees multiply to {n}, not {cfg['num_gpus']} GPUs"
    return None


@register_prune
def prune_by_memory_estimation(tuner_cfg, cfg):
    limit = float(tuner_cfg.get('max_mem_usage', 288.0))
    est = estimate_memory_gb(tuner_cfg['model_cfg'], cfg)
    cfg['estimated_memory_usage'] = round(est, 2)
    if est > limit:
        return f"estimated {est:.1f} GB > {limit:.0f} GB"
    return None


def _same_but(cfg, other, keys):
    for k in ('dp_degree', 'mp_degree', 'pp_degree', 'vpp_degree', 'sharding_degree', 'sharding_stage',
              'micro_batch_size', 'use_recompute', 'recompute_granularity'):
        if k not in keys and cfg.get(k) != other.get(k):
            return False
    return True


_RECOMP_LEVEL = {None: 0, 'core_attn': 1, 'full_attn': 2, 'full': 3}


@register_prune_history
def prune_by_mbs_history(tuner_cfg, cfg, history):
    """A smaller micro batch of the same layout ran out of memory: so will this one."""
    for h in history:
        if h.get('oom') and _same_but(cfg, h, ('micro_batch_size', 'acc_steps')) and \
                h['micro_batch_size'] <= cfg['micro_batch_size']:
            return f"micro batch {h['micro_batch_size']} of this layout ran out of memory"
    return None


@register_prune_history
def prune_by_recompute_history(tuner_cfg, cfg, history):
    """Less recomputation of the same layout fit: recomputing more only costs time; more
    recomputation of the same layout ran out of memory: less will too."""
    mine = _RECOMP_LEVEL[cfg.get('recompute_granularity') if cfg.get('use_recompute') else None]
    for h in history:
        if not _same_but(cfg, h, ('use_recompute', 'recompute_granularity')):
            continue
        lvl = _RECOMP_LEVEL[h.get('recompute_granularity') if h.get('use_recompute') else None]
        if not h.get('oom') and h.get('time', -1) != -1 and lvl < mine:
            return "a lighter recompute of this layout fit in memory"
        if h.get('oom') and lvl >= mine:
            return "a heavier recompute of this layout ran out of memory"
    return None


def prune(tuner_cfg, cfg, history=()):
    """First reason ``cfg`` is pruned (None: run it)."""
    for fn in _RULES:
        r = fn(tuner_cfg, cfg)
        if r:
            return r
    for fn in _HISTORY_RULES:
        r = fn(tuner_cfg, cfg, list(history))
        if r:
            return r
    return None
