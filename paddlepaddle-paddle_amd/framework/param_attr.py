"""paddle.ParamAttr / WeightNormParamAttr (reference: python/paddle/base/param_attr.py)."""


class ParamAttr:
    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None, trainable=True,
                 do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if arg is False:
            return False
        from ..nn.initializer import Initializer
        if isinstance(arg, Initializer):
            return ParamAttr(initializer=arg)
        if isinstance(arg, (list, tuple)):
            return [ParamAttr._to_attr(a) for a in arg]
        raise TypeError(f"{type(arg)} cannot be cast to ParamAttr")


class WeightNormParamAttr(ParamAttr):
    def __init__(self, dim=None, **kw):
        super().__init__(**kw)
        self.dim = dim
