"""Per-GPU memory model of a decoder-only transformer under hybrid parallelism (reference:
python/paddle/distributed/auto_tuner/memory_cost_model.py and cost_model.py get_mem).

Terms (GB, per GPU):
* parameters — bf16, the stage's layers split over mp (and over sharding at stage 3); the
  embedding / LM head (tied) on the first and last stage, split over mp;
* gradients — bf16 (fp32 when ``main_grad``), split over sharding from stage 2;
* optimizer state — fp32 master + Adam moments = 12 B per parameter, split over sharding from
  stage 1;
* activations — per layer and micro-batch ``s*b*h*(34/mp)`` bytes with flash attention (no
  materialised scores: the 5*a*s/h term of Korthikanti et al. is gone), ``2*s*b*h`` with full
  recompute (only the layer input is kept), about half of the full set for 'full_attn'; 1F1B keeps
  up to ``pp`` micro-batches of the first stage's layers in flight;
* workspace — kernel scratch + allocator slack (``workspace_gb``, 6 GB default).
"""


def model_dims(model_cfg):
    h = int(model_cfg['hidden_size'])
    return dict(h=h, L=int(model_cfg['num_layers']), a=int(model_cfg['num_attention_heads']),
                V=int(model_cfg.get('vocab_size', 50304)), s=int(model_cfg.get('seq_length', 1024)),
                f=int(model_cfg.get('intermediate_size', 4 * h)))


def layer_params(d):
    """Parameters of one decoder layer (qkv + out projections, the FFN, two norms, biases)."""
    h, f = d['h'], d['f']
    return 4 * h * h + 2 * h * f + 9 * h + f


def total_params(d):
    return d['L'] * layer_params(d) + d['V'] * d['h'] + d['s'] * d['h']


def estimate_memory_gb(model_cfg, cfg, workspace_gb=6.0, main_grad=False):
    """Peak memory (GB) of one GPU for a candidate ``cfg`` (dp/mp/pp/vpp/sharding degrees,
    sharding_stage, micro_batch_size, use_recompute, recompute_granularity, acc_steps)."""
    d = model_dims(model_cfg)
    mp, pp = int(cfg.get('mp_degree', 1)), int(cfg.get('pp_degree', 1))
    sh, stage = int(cfg.get('sharding_degree', 1)), int(cfg.get('sharding_stage', 1) or 1)
    b = int(cfg.get('micro_batch_size', 1))
    acc = int(cfg.get('acc_steps', 1))
    h, L, s = d['h'], d['L'], d['s']
    p_layers = L * layer_params(d) / (mp * pp)
    p_emb = (d['V'] * h / mp) + s * h          # first / last stage: embedding (tied LM head)
    p = p_layers + p_emb
    shard_p = sh if stage >= 3 else 1
    shard_g = sh if stage >= 2 else 1
    shard_o = sh if sh > 1 else 1
    params = 2 * p / shard_p
    grads = (4 if main_grad else 2) * p / shard_g
    opt = 12 * p / shard_o
    if stage >= 3 and sh > 1:
        params += 2 * (p_layers / max(L // pp, 1)) * 2  # two layers gathered at a time (prefetch)
    gran = cfg.get('recompute_granularity') if cfg.get('use_recompute') else None
    per_layer = s * b * h * 34 / mp
    if gran == 'full':
        per_layer = 2 * s * b * h
    elif gran == 'full_attn':
        per_layer = s * b * h * 18 / mp
    elif gran == 'core_attn':
        per_layer = s * b * h * 30 / mp
    inflight = min(pp, acc) if pp > 1 else 1
    acts = per_layer * (L / pp) * inflight
    # the LM head's logits (bf16 + fp32 softmax) of the last stage
    logits = s * b * d['V'] / mp * 6
    total = params + grads + opt + acts + logits
    return total / 1e9 + workspace_gb
