"""AMP op lists (reference: python/paddle/amp/amp_lists.py)."""
WHITE_LIST = {'conv2d', 'matmul', 'matmul_v2', 'mul', 'einsum', 'linear', 'flash_attn', 'bmm', 'conv3d'}
BLACK_LIST = {'exp', 'square', 'log', 'mean', 'sum', 'cos_sim', 'softmax_with_cross_entropy', 'sigmoid_cross_entropy_with_logits',
              'c_softmax_with_cross_entropy', 'cross_entropy', 'cross_entropy2', 'reduce_sum', 'layer_norm', 'batch_norm'}


def white_list():
    return {'float16': {'O1': set(WHITE_LIST), 'O2': set(WHITE_LIST)},
            'bfloat16': {'O1': set(WHITE_LIST), 'O2': set(WHITE_LIST)}}


def black_list():
    return {'float16': {'O1': set(BLACK_LIST), 'O2': set(BLACK_LIST)},
            'bfloat16': {'O1': set(BLACK_LIST), 'O2': set(BLACK_LIST)}}
