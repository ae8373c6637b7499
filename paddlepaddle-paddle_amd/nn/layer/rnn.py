"""Recurrent layers (reference: python/paddle/nn/layer/rnn.py).

Parameter names/layouts follow the reference (``weight_ih_l{k}[_reverse]`` of shape
[gates*hidden, input]); the multi-layer fused path runs MIOpen RNN kernels through the
storage layer's ``_VF`` entry points with our parameters as the flat weight list.
"""
import math

import torch

from .layers import Layer
from .. import initializer as I
from ...core.tensor import Tensor, _wrap, _unwrap


class RNNCellBase(Layer):
    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        b = _unwrap(batch_ref).shape[batch_dim_idx]
        t = _unwrap(batch_ref)
        z = torch.full((b, self.hidden_size), init_value, dtype=t.dtype, device=t.device)
        if isinstance(self, LSTMCell):
            return _wrap(z), _wrap(z.clone())
        return _wrap(z)


def _cell_params(self, input_size, hidden_size, gates, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr):
    std = 1.0 / math.sqrt(hidden_size)
    init = I.Uniform(-std, std)
    self.weight_ih = self.create_parameter([gates * hidden_size, input_size], weight_ih_attr, default_initializer=init)
    self.weight_hh = self.create_parameter([gates * hidden_size, hidden_size], weight_hh_attr, default_initializer=init)
    self.bias_ih = self.create_parameter([gates * hidden_size], bias_ih_attr, is_bias=True, default_initializer=init)
    self.bias_hh = self.create_parameter([gates * hidden_size], bias_hh_attr, is_bias=True, default_initializer=init)


class SimpleRNNCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        self.input_size, self.hidden_size, self.activation = input_size, hidden_size, activation
        _cell_params(self, input_size, hidden_size, 1, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        fn = torch.rnn_tanh_cell if self.activation == 'tanh' else torch.rnn_relu_cell
        h = fn(_unwrap(inputs), _unwrap(states), self.weight_ih._t, self.weight_hh._t,
               None if self.bias_ih is None else self.bias_ih._t, None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), _wrap(h)

    @property
    def state_shape(self):
        return (self.hidden_size,)


class LSTMCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, proj_size=0, name=None):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        _cell_params(self, input_size, hidden_size, 4, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h, c = torch.lstm_cell(_unwrap(inputs), (_unwrap(states[0]), _unwrap(states[1])), self.weight_ih._t,
                               self.weight_hh._t, None if self.bias_ih is None else self.bias_ih._t,
                               None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), (_wrap(h), _wrap(c))

    @property
    def state_shape(self):
        return ((self.hidden_size,), (self.hidden_size,))


class GRUCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        _cell_params(self, input_size, hidden_size, 3, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h = torch.gru_cell(_unwrap(inputs), _unwrap(states), self.weight_ih._t, self.weight_hh._t,
                           None if self.bias_ih is None else self.bias_ih._t,
                           None if self.bias_hh is None else self.bias_hh._t)
        return _wrap(h), _wrap(h)

    @property
    def state_shape(self):
        return (self.hidden_size,)


class RNN(Layer):
    """Unrolls any cell over time (reference RNN wrapper)."""

    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell, self.is_reverse, self.time_major = cell, is_reverse, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        x = _unwrap(inputs)
        if not self.time_major:
            x = x.transpose(0, 1)
        T = x.shape[0]
        states = initial_states
        if states is None:
            states = self.cell.get_initial_states(_wrap(x[0]))
        outs = []
        steps = range(T - 1, -1, -1) if self.is_reverse else range(T)
        seq = _unwrap(sequence_length) if sequence_length is not None else None
        for t in steps:
            y, new_states = self.cell(_wrap(x[t]), states, **kwargs)
            if seq is not None:
                keep = (t < seq).to(x.dtype).unsqueeze(-1)
                def _mix(n, o):
                    return _wrap(_unwrap(n) * keep + _unwrap(o) * (1 - keep))
                new_states = tuple(_mix(n, o) for n, o in zip(new_states, states)) if isinstance(new_states, tuple) \
                    else _mix(new_states, states)
                y = _wrap(_unwrap(y) * keep)
            states = new_states
            outs.append(_unwrap(y))
        if self.is_reverse:
            outs = outs[::-1]
        out = torch.stack(outs, 0)
        if not self.time_major:
            out = out.transpose(0, 1)
        return _wrap(out), states


class BiRNN(Layer):
    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.rnn_fw = RNN(cell_fw, False, time_major)
        self.rnn_bw = RNN(cell_bw, True, time_major)

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        s_fw, s_bw = (None, None) if initial_states is None else initial_states
        o_fw, st_fw = self.rnn_fw(inputs, s_fw, sequence_length, **kwargs)
        o_bw, st_bw = self.rnn_bw(inputs, s_bw, sequence_length, **kwargs)
        return _wrap(torch.cat([_unwrap(o_fw), _unwrap(o_bw)], -1)), (st_fw, st_bw)


class _RNNBase(Layer):
    _mode = 'RNN_TANH'
    _gates = 1

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, activation=None,
                 proj_size=0, name=None):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.direction = direction
        self.num_directions = 2 if direction in ('bidirect', 'bidirectional') else 1
        self.time_major, self.dropout = time_major, dropout
        if activation == 'relu':
            self._mode = 'RNN_RELU'
        std = 1.0 / math.sqrt(hidden_size)
        init = I.Uniform(-std, std)
        G = self._gates
        self._flat_names = []
        for layer in range(num_layers):
            for d in range(self.num_directions):
                sfx = f"_l{layer}" + ("_reverse" if d == 1 else "")
                in_sz = input_size if layer == 0 else hidden_size * self.num_directions
                for n, shp, attr, is_b in (("weight_ih", [G * hidden_size, in_sz], weight_ih_attr, False),
                                           ("weight_hh", [G * hidden_size, hidden_size], weight_hh_attr, False),
                                           ("bias_ih", [G * hidden_size], bias_ih_attr, True),
                                           ("bias_hh", [G * hidden_size], bias_hh_attr, True)):
                    p = self.create_parameter(shp, attr, is_bias=is_b, default_initializer=init)
                    setattr(self, n + sfx, p)
                    self._flat_names.append(n + sfx)

    def flatten_parameters(self):
        pass

    def forward(self, inputs, initial_states=None, sequence_length=None):
        x = _unwrap(inputs)
        batch_first = not self.time_major
        B = x.shape[0] if batch_first else x.shape[1]
        L = self.num_layers * self.num_directions
        weights = [getattr(self, n)._t for n in self._flat_names]
        bidir = self.num_directions == 2
        if initial_states is None:
            z = torch.zeros(L, B, self.hidden_size, dtype=x.dtype, device=x.device)
            initial_states = (z, z.clone()) if self._mode == 'LSTM' else z
        elif isinstance(initial_states, (tuple, list)):
            initial_states = tuple(_unwrap(s) for s in initial_states)
        else:
            initial_states = _unwrap(initial_states)
        if sequence_length is not None:
            lens = _unwrap(sequence_length).cpu()
            x = torch.nn.utils.rnn.pack_padded_sequence(x, lens, batch_first=batch_first, enforce_sorted=False)
        mod = {'LSTM': torch.nn.LSTM, 'GRU': torch.nn.GRU}.get(self._mode)
        if self._mode == 'LSTM':
            if sequence_length is None:
                out, h, c = torch._VF.lstm(x, initial_states, weights, True, self.num_layers, self.dropout,
                                           self.training, bidir, batch_first)
            else:
                out, (h, c) = _packed(torch.nn.LSTM, self, x, initial_states, weights, bidir, batch_first)
            state = (_wrap(h), _wrap(c))
        elif self._mode == 'GRU':
            out, h = torch._VF.gru(x, initial_states, weights, True, self.num_layers, self.dropout, self.training,
                                   bidir, batch_first) if sequence_length is None else \
                _packed(torch.nn.GRU, self, x, initial_states, weights, bidir, batch_first)
            state = _wrap(h)
        else:
            fn = torch._VF.rnn_tanh if self._mode == 'RNN_TANH' else torch._VF.rnn_relu
            out, h = fn(x, initial_states, weights, True, self.num_layers, self.dropout, self.training, bidir,
                        batch_first) if sequence_length is None else \
                _packed(torch.nn.RNN, self, x, initial_states, weights, bidir, batch_first)
            state = _wrap(h)
        if sequence_length is not None:
            out, _ = torch.nn.utils.rnn.pad_packed_sequence(out, batch_first=batch_first)
        _ = mod
        return _wrap(out), state


def _packed(cls, self, packed, hx, weights, bidir, batch_first):
    kw = {}
    if cls is torch.nn.RNN:
        kw['nonlinearity'] = 'tanh' if self._mode == 'RNN_TANH' else 'relu'
    m = cls(self.input_size, self.hidden_size, self.num_layers, bias=True, batch_first=batch_first,
            dropout=self.dropout, bidirectional=bidir, **kw)
    m.to(weights[0].device)
    for name, w in zip(m._flat_weights_names, weights):
        setattr(m, name, torch.nn.Parameter(w)) if False else None
    m._flat_weights = list(weights)
    return m(packed, hx)


class SimpleRNN(_RNNBase):
    _mode, _gates = 'RNN_TANH', 1


class LSTM(_RNNBase):
    _mode, _gates = 'LSTM', 4


class GRU(_RNNBase):
    _mode, _gates = 'GRU', 3
