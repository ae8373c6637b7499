"""Loss layers (reference: python/paddle/nn/layer/loss.py)."""
from .layers import Layer
from .. import functional as F


class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction='mean', soft_label=False, axis=-1, use_softmax=True,
                 label_smoothing=0.0, name=None):
        super().__init__()
        self.weight, self.ignore_index, self.reduction = weight, ignore_index, reduction
        self.soft_label, self.axis, self.use_softmax, self.label_smoothing = soft_label, axis, use_softmax, label_smoothing

    def forward(self, input, label):  # noqa: A002
        return F.cross_entropy(input, label, self.weight, self.ignore_index, self.reduction, self.soft_label,
                               self.axis, self.use_softmax, self.label_smoothing)


def _loss_cls(name, fn, argnames, defaults, nin=2):
    def __init__(self, *args, **kwargs):
        Layer.__init__(self)
        vals = dict(zip(argnames, defaults))
        vals.update(dict(zip(argnames, args)))
        vals.update({k: v for k, v in kwargs.items() if k != 'name'})
        self._kw = vals

    def forward(self, *inputs):
        return fn(*inputs, **self._kw)
    return type(name, (Layer,), {'__init__': __init__, 'forward': forward})


MSELoss = _loss_cls('MSELoss', F.mse_loss, ['reduction'], ['mean'])
L1Loss = _loss_cls('L1Loss', F.l1_loss, ['reduction'], ['mean'])
SmoothL1Loss = _loss_cls('SmoothL1Loss', F.smooth_l1_loss, ['reduction', 'delta'], ['mean', 1.0])
BCELoss = _loss_cls('BCELoss', F.binary_cross_entropy, ['weight', 'reduction'], [None, 'mean'])
BCEWithLogitsLoss = _loss_cls('BCEWithLogitsLoss', F.binary_cross_entropy_with_logits,
                              ['weight', 'reduction', 'pos_weight'], [None, 'mean', None])
NLLLoss = _loss_cls('NLLLoss', F.nll_loss, ['weight', 'ignore_index', 'reduction'], [None, -100, 'mean'])
KLDivLoss = _loss_cls('KLDivLoss', F.kl_div, ['reduction', 'log_target'], ['mean', False])
MarginRankingLoss = _loss_cls('MarginRankingLoss', F.margin_ranking_loss, ['margin', 'reduction'], [0.0, 'mean'])
HingeEmbeddingLoss = _loss_cls('HingeEmbeddingLoss', F.hinge_embedding_loss, ['margin', 'reduction'], [1.0, 'mean'])
CosineEmbeddingLoss = _loss_cls('CosineEmbeddingLoss', F.cosine_embedding_loss, ['margin', 'reduction'], [0, 'mean'])
TripletMarginLoss = _loss_cls('TripletMarginLoss', F.triplet_margin_loss,
                              ['margin', 'p', 'epsilon', 'swap', 'reduction'], [1.0, 2, 1e-6, False, 'mean'])
TripletMarginWithDistanceLoss = _loss_cls('TripletMarginWithDistanceLoss', F.triplet_margin_with_distance_loss,
                                          ['distance_function', 'margin', 'swap', 'reduction'],
                                          [None, 1.0, False, 'mean'])
MultiLabelSoftMarginLoss = _loss_cls('MultiLabelSoftMarginLoss', F.multi_label_soft_margin_loss,
                                     ['weight', 'reduction'], [None, 'mean'])
MultiMarginLoss = _loss_cls('MultiMarginLoss', F.multi_margin_loss, ['p', 'margin', 'weight', 'reduction'],
                            [1, 1.0, None, 'mean'])
SoftMarginLoss = _loss_cls('SoftMarginLoss', F.soft_margin_loss, ['reduction'], ['mean'])
PoissonNLLLoss = _loss_cls('PoissonNLLLoss', F.poisson_nll_loss, ['log_input', 'full', 'epsilon', 'reduction'],
                           [True, False, 1e-8, 'mean'])
GaussianNLLLoss = _loss_cls('GaussianNLLLoss', F.gaussian_nll_loss, ['full', 'epsilon', 'reduction'],
                            [False, 1e-6, 'mean'])
CTCLoss = _loss_cls('CTCLoss', F.ctc_loss, ['blank', 'reduction'], [0, 'mean'])
RNNTLoss = _loss_cls('RNNTLoss', F.rnnt_loss, ['blank', 'fastemit_lambda', 'reduction'], [0, 0.001, 'mean'])


class HSigmoidLoss(Layer):
    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None, is_custom=False, is_sparse=False,
                 name=None):
        super().__init__()
        self._num_classes = num_classes
        self.weight = self.create_parameter([num_classes - 1, feature_size], attr=weight_attr)
        self.bias = self.create_parameter([num_classes - 1, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):  # noqa: A002
        return F.hsigmoid_loss(input, label, self._num_classes, self.weight, self.bias, path_table, path_code)


class AdaptiveLogSoftmaxWithLoss(Layer):
    """Reference nn/layer/loss.py AdaptiveLogSoftmaxWithLoss: head Linear(in, shortlist + n_clusters)
    and per cluster i a (Linear(in, in // div_value**(i+1)), Linear(.., cluster size)) tail."""

    def __init__(self, in_features, n_classes, cutoffs, div_value=4.0, head_bias=False, name=None):
        super().__init__()
        cutoffs = list(cutoffs)
        if len(cutoffs) == 0 or cutoffs != sorted(cutoffs) or min(cutoffs) <= 0 or max(cutoffs) > n_classes - 1 \
                or len(set(cutoffs)) != len(cutoffs):
            raise ValueError("cutoffs should be a sorted list of unique positive ints < n_classes - 1")
        self.in_features, self.n_classes, self.div_value = in_features, n_classes, div_value
        self.cutoffs = cutoffs + [n_classes]
        self.shortlist_size = self.cutoffs[0]
        self.n_clusters = len(self.cutoffs) - 1
        self.head_size = self.shortlist_size + self.n_clusters
        self.head_weight = self.create_parameter([in_features, self.head_size])
        self.head_bias = self.create_parameter([self.head_size], is_bias=True) if head_bias else None
        self.tail_weights = []
        for i in range(self.n_clusters):
            hsz = int(in_features // (div_value ** (i + 1)))
            osz = self.cutoffs[i + 1] - self.cutoffs[i]
            w0 = self.create_parameter([in_features, hsz])
            w1 = self.create_parameter([hsz, osz])
            self.add_parameter(f'tail_{i}_0', w0)
            self.add_parameter(f'tail_{i}_1', w1)
            self.tail_weights.append([w0, w1])

    def forward(self, input, label):  # noqa: A002
        return F.adaptive_log_softmax_with_loss(input, label, self.head_weight, self.tail_weights, self.cutoffs,
                                                self.head_bias)

    def log_prob(self, input):  # noqa: A002
        import torch
        from ...core.tensor import _wrap
        x = input._t
        head = x @ self.head_weight._t
        if self.head_bias is not None:
            head = head + self.head_bias._t
        hl = torch.log_softmax(head, -1)
        parts = [hl[:, :self.shortlist_size]]
        for i, (w0, w1) in enumerate(self.tail_weights):
            parts.append(torch.log_softmax((x @ w0._t) @ w1._t, -1) + hl[:, self.shortlist_size + i:self.shortlist_size + i + 1])
        return _wrap(torch.cat(parts, -1))

    def predict(self, input):  # noqa: A002
        return self.log_prob(input).argmax(-1)