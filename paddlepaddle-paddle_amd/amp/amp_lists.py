"""AMP op lists (reference: python/paddle/amp/amp_lists.py).

Op names are the reference's operator names; the dygraph ops carrying them are tagged with
``core.amp_dispatch.amp_op``.  Level semantics: OD = white list only (empty black list),
O1 = white + full black list, O2 = white + the "extra" black list (pure low precision).
"""
WHITE_LIST = {
    'conv2d', 'einsum', 'matmul', 'matmul_v2', 'max_pool2d_with_index', 'mul', 'fused_gemm_epilogue',
    'fused_rotary_position_embedding', 'flash_attn',
}

ONLY_FP16_WHITE_LIST = {
    'fake_quantize_dequantize_abs_max', 'fake_quantize_dequantize_moving_average_abs_max', 'fused_attention',
    'fused_feedforward',
}

FP16_WHITE_LIST = WHITE_LIST | ONLY_FP16_WHITE_LIST

FP16_BLACK_LIST = {
    'tan', 'acos', 'asin', 'sinh', 'cosh', 'atanh', 'tanh_shrink', 'erfinv', 'exp', 'expm1', 'log', 'log10', 'log2',
    'reciprocal', 'rsqrt', 'pow', 'square', 'reduce_sum', 'mean', 'reduce_mean', 'reduce_prod', 'cumprod', 'cumsum',
    'dist', 'pnorm', 'frobenius_norm', 'renorm', 'group_norm', 'layer_norm', 'softmax', 'softmin', 'softplus',
    'log_softmax', 'softmax_with_cross_entropy', 'sigmoid_cross_entropy_with_logits', 'c_softmax_with_cross_entropy',
    'cross_entropy', 'cross_entropy2', 'nll_loss', 'huber_loss', 'triplet_margin_loss', 'log_loss', 'hsigmoid_loss',
    'margin_cross_entropy',
}

EXTRA_BLACK_LIST = {
    'linear_interp_v2', 'nearest_interp_v2', 'bilinear_interp_v2', 'bicubic_interp_v2', 'trilinear_interp_v2',
    'lookup_table', 'lookup_table_v2', 'scatter',
}

BF16_WHITE_LIST = WHITE_LIST
BF16_BLACK_LIST = FP16_BLACK_LIST


def white_list():
    return {
        'float16': {'OD': set(FP16_WHITE_LIST), 'O1': set(FP16_WHITE_LIST), 'O2': set(FP16_WHITE_LIST)},
        'bfloat16': {'OD': set(BF16_WHITE_LIST), 'O1': set(BF16_WHITE_LIST), 'O2': set(BF16_WHITE_LIST)},
    }


def black_list():
    return {
        'float16': {'OD': set(), 'O1': FP16_BLACK_LIST | EXTRA_BLACK_LIST, 'O2': set(EXTRA_BLACK_LIST)},
        'bfloat16': {'OD': set(), 'O1': BF16_BLACK_LIST | EXTRA_BLACK_LIST, 'O2': set(EXTRA_BLACK_LIST)},
    }


def _update_list(custom_white_list, custom_black_list, level='O1', dtype='float16'):
    """Default lists for (level, dtype) with the custom lists applied (reference auto_cast.py _update_list)."""
    if level == 'O0':
        return set(), set()
    d = 'bfloat16' if 'bf' in str(dtype) else 'float16'
    lv = level if level in ('OD', 'O1', 'O2') else 'O1'
    wl = set(white_list()[d][lv])
    bl = set(black_list()[d][lv])
    if custom_white_list and custom_black_list:
        both = set(custom_white_list) & set(custom_black_list)
        if both:
            raise ValueError(f"Custom white list overlaps custom black list: {sorted(both)}")
    for op in custom_white_list or ():
        wl.add(op)
        bl.discard(op)
    for op in custom_black_list or ():
        bl.add(op)
        wl.discard(op)
    return wl, bl
