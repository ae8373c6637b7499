"""Analytic step-time model of a hybrid-parallel transformer step on MI355X nodes (the ranking the
``cost_model`` search uses; reference role: python/paddle/distributed/auto_tuner/cost_model.py).

Hardware constants are this framework's own measurements on MI355X (round 5/6 profiles):
* dense bf16 MFMA: 2.5 PF/s spec; the hand-written GEMMs hold 1.2-1.4 PF/s on GPT-3 1.3B shapes
  and the whole GPT step about 45 % of spec — ``mfu`` 0.45 at full-size per-GPU GEMMs, falling off
  as tensor parallelism / small micro-batches shrink them (``_gemm_eff``);
* xGMI: 7 links x ~64 GB/s usable per direction per GPU inside a node — a ring collective over g
  GPUs runs on ``min(g - 1, 7)`` link pairs; between nodes ``inter_node_gbps`` (RoCE/IB, 50 GB/s);
* data-parallel / sharding gradient collectives overlap backward except for ``dp_exposed`` (30 %).
"""
from .memory_cost_model import model_dims, layer_params

PEAK = 2.5e15
LINK_GBPS = 64.0
INTER_NODE_GBPS = 50.0


def _gemm_eff(rows, cols, mfu):
    """MFU of the step's GEMMs when each is [rows x cols]-sized per GPU."""
    small = min(1.0, rows / 8192.0) ** 0.25 * min(1.0, cols / 2048.0) ** 0.25
    return mfu * small


def _ring_bw(g, gpus_per_node, intra=True):
    if g <= 1:
        return float('inf')
    if not intra:
        return INTER_NODE_GBPS * 1e9
    return min(g - 1, 7) * LINK_GBPS * 1e9


def _allreduce_s(nbytes, g, bw):
    return 0.0 if g <= 1 else 2.0 * (g - 1) / g * nbytes / bw


def estimate_step_time(model_cfg, cfg, num_gpus, gpus_per_node=8, mfu=0.45, dp_exposed=0.3):
    """Estimated seconds per global step of candidate ``cfg``."""
    d = model_dims(model_cfg)
    h, L, s, V = d['h'], d['L'], d['s'], d['V']
    dp, mp, pp = int(cfg.get('dp_degree', 1)), int(cfg.get('mp_degree', 1)), int(cfg.get('pp_degree', 1))
    vpp, sh = int(cfg.get('vpp_degree', 1) or 1), int(cfg.get('sharding_degree', 1))
    stage = int(cfg.get('sharding_stage', 1) or 1)
    b, acc = int(cfg.get('micro_batch_size', 1)), int(cfg.get('acc_steps', 1))
    gbs = int(model_cfg.get('global_batch_size', b * acc * dp * sh))
    tokens = gbs * s
    p = L * layer_params(d) + V * h
    flops = 6.0 * p * tokens + 6.0 * L * s * h * tokens  # GEMMs + causal attention
    gran = cfg.get('recompute_granularity') if cfg.get('use_recompute') else None
    if gran == 'full':
        flops *= 4.0 / 3.0
    elif gran == 'full_attn':
        flops *= 1.15
    elif gran == 'core_attn':
        flops *= 1.04
    eff = _gemm_eff(b * s, max(h // mp, 1), mfu)
    compute = flops / num_gpus / (PEAK * eff)
    # pipeline bubble (1F1B / interleaved)
    if pp > 1:
        compute *= 1.0 + (pp - 1) / (vpp * acc)
    # tensor parallel: 2 all-reduces of [b, s, h] per layer forward, 2 backward, per micro-batch
    intra_mp = mp <= gpus_per_node
    tp = 4 * (L / pp) * acc * _allreduce_s(2.0 * b * s * h, mp, _ring_bw(mp, gpus_per_node, intra_mp))
    # pipeline sends: activations forward, gradients backward, per micro-batch and stage boundary
    pp_comm = 0.0
    if pp > 1:
        pp_comm = 2 * acc * vpp * (2.0 * b * s * h) / (LINK_GBPS * 1e9)
    # data parallel + sharding: gradient reduce (+ parameter gathers at stage 3)
    p_gpu = p / (mp * pp)
    g = dp * sh
    intra_dp = g * mp * pp <= gpus_per_node
    bw = _ring_bw(g, gpus_per_node, intra_dp)
    dp_s = _allreduce_s(2.0 * p_gpu, g, bw)
    if sh > 1 and stage >= 3:
        dp_s *= 2.0  # forward / backward parameter all-gathers on top of the reduce-scatter
    return compute + tp + pp_comm + dp_exposed * dp_s
