"""Containers (reference: python/paddle/nn/layer/container.py)."""
import collections

from .layers import Layer
from ...core.tensor import Parameter


class Sequential(Layer):
    def __init__(self, *layers):
        super().__init__()
        if len(layers) > 0 and isinstance(layers[0], (list, tuple)) and len(layers[0]) == 2 and isinstance(layers[0][0], str):
            for name, layer in layers:
                self.add_sublayer(name, layer)
        elif len(layers) == 1 and isinstance(layers[0], collections.OrderedDict):
            for name, layer in layers[0].items():
                self.add_sublayer(name, layer)
        else:
            for i, layer in enumerate(layers):
                self.add_sublayer(str(i), layer)

    def __getitem__(self, name):
        if isinstance(name, slice):
            return self.__class__(*(list(self._sub_layers.values())[name]))
        if isinstance(name, str):
            return self._sub_layers[name]
        if name < 0:
            name += len(self._sub_layers)
        return list(self._sub_layers.values())[name]

    def __setitem__(self, name, layer):
        self._sub_layers[str(name)] = layer

    def __delitem__(self, name):
        del self._sub_layers[str(name)]

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers.values())

    def append(self, layer):
        self.add_sublayer(str(len(self)), layer)
        return self

    def forward(self, input):  # noqa: A002
        for layer in self._sub_layers.values():
            input = layer(input)
        return input


class LayerList(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            for i, l in enumerate(sublayers):
                self.add_sublayer(str(i), l)

    def _abs(self, idx):
        if idx < 0:
            idx += len(self)
        return idx

    def __getitem__(self, idx):
        if isinstance(idx, slice):
            return self.__class__(list(self._sub_layers.values())[idx])
        return self._sub_layers[str(self._abs(idx))]

    def __setitem__(self, idx, layer):
        self._sub_layers[str(self._abs(idx))] = layer

    def __delitem__(self, idx):
        if isinstance(idx, slice):
            keys = list(self._sub_layers.keys())[idx]
            for k in keys:
                del self._sub_layers[k]
        else:
            del self._sub_layers[str(self._abs(idx))]
        vals = list(self._sub_layers.values())
        self._sub_layers.clear()
        for i, v in enumerate(vals):
            self._sub_layers[str(i)] = v

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers.values())

    def append(self, sublayer):
        self.add_sublayer(str(len(self)), sublayer)
        return self

    def insert(self, index, sublayer):
        vals = list(self._sub_layers.values())
        vals.insert(index, sublayer)
        self._sub_layers.clear()
        for i, v in enumerate(vals):
            self._sub_layers[str(i)] = v

    def extend(self, sublayers):
        for l in sublayers:
            self.append(l)
        return self


class LayerDict(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            self.update(sublayers)

    def __getitem__(self, key):
        return self._sub_layers[key]

    def __setitem__(self, key, layer):
        self.add_sublayer(key, layer)

    def __delitem__(self, key):
        del self._sub_layers[key]

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers)

    def __contains__(self, key):
        return key in self._sub_layers

    def clear(self):
        self._sub_layers.clear()

    def pop(self, key):
        return self._sub_layers.pop(key)

    def keys(self):
        return self._sub_layers.keys()

    def items(self):
        return self._sub_layers.items()

    def values(self):
        return self._sub_layers.values()

    def update(self, sublayers):
        items = sublayers.items() if hasattr(sublayers, 'items') else sublayers
        for k, v in items:
            self.add_sublayer(k, v)


class ParameterList(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters is not None:
            for i, p in enumerate(parameters):
                self.add_parameter(str(i), p)

    def __getitem__(self, idx):
        if idx < 0:
            idx += len(self)
        return self._parameters[str(idx)]

    def __setitem__(self, idx, param):
        self._parameters[str(idx)] = param

    def __len__(self):
        return len(self._parameters)

    def __iter__(self):
        return iter(self._parameters.values())

    def append(self, parameter):
        self.add_parameter(str(len(self)), parameter)
        return self


class ParameterDict(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters is not None:
            for k, v in (parameters.items() if hasattr(parameters, 'items') else parameters):
                self.add_parameter(k, v)

    def __getitem__(self, k):
        return self._parameters[k]

    def __setitem__(self, k, v):
        self.add_parameter(k, v)

    def __len__(self):
        return len(self._parameters)

    def __iter__(self):
        return iter(self._parameters)

    def keys(self):
        return self._parameters.keys()

    def items(self):
        return self._parameters.items()

    def values(self):
        return self._parameters.values()


_ = Parameter
