"""paddle.regularizer (reference: python/paddle/regularizer.py)."""


class WeightDecayRegularizer:
    def __init__(self, coeff=0.0):
        self._coeff = float(coeff)

    def __repr__(self):
        return f"{self.__class__.__name__}(coeff={self._coeff})"


class L1Decay(WeightDecayRegularizer):
    pass


class L2Decay(WeightDecayRegularizer):
    pass
