from .mp_layers import VocabParallelEmbedding, ColumnParallelLinear, RowParallelLinear, ParallelCrossEntropy  # noqa: F401
from .mp_ops import _c_identity, _mp_allreduce, _c_split, _c_concat, _c_softmax_with_cross_entropy  # noqa: F401
from .random import RNGStatesTracker, get_rng_state_tracker, model_parallel_random_seed  # noqa: F401


def _split_api(x, size, operation, axis=0, num_partitions=1, gather_out=True, weight_attr=None, bias_attr=None,
               name=None):
    """paddle.distributed.split: build (and apply) a model-parallel linear / embedding."""
    if operation == 'embedding':
        layer = VocabParallelEmbedding(size[0], size[1], weight_attr=weight_attr)
    elif axis == 1:
        layer = ColumnParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                     gather_output=gather_out)
    else:
        layer = RowParallelLinear(size[0], size[1], weight_attr=weight_attr, has_bias=bias_attr is not False,
                                  input_is_parallel=False)
    return layer(x)
