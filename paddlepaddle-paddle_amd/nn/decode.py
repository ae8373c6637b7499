"""Beam search decoding (reference: python/paddle/nn/decode.py: BeamSearchDecoder, dynamic_decode)."""
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


class Decoder:
    def initialize(self, inits):
        raise NotImplementedError

    def step(self, time, inputs, states, **kwargs):
        raise NotImplementedError

    def finalize(self, outputs, final_states, sequence_lengths):
        raise NotImplementedError

    @property
    def tracks_own_finished(self):
        return False


class BeamSearchDecoder(Decoder):
    """Beam search over a cell: state tensors are tiled to [batch*beam, ...]."""

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None, output_fn=None):
        self.cell, self.start_token, self.end_token = cell, start_token, end_token
        self.beam_size, self.embedding_fn, self.output_fn = beam_size, embedding_fn, output_fn

    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        t = _unwrap(x)
        t = t.unsqueeze(1).expand(t.shape[0], beam_size, *t.shape[1:])
        return _wrap(t.reshape(-1, *t.shape[2:]))

    def _map(self, fn, s):
        if isinstance(s, (tuple, list)):
            return type(s)(self._map(fn, e) for e in s)
        return fn(s)

    def initialize(self, initial_cell_states):
        first = initial_cell_states
        while isinstance(first, (tuple, list)):
            first = first[0]
        B = _unwrap(first).shape[0]
        K = self.beam_size
        dev = _unwrap(first).device
        self.batch_size = B
        states = self._map(lambda s: self.tile_beam_merge_with_batch(s, K), initial_cell_states)
        log_probs = torch.full((B, K), float('-inf'), device=dev)
        log_probs[:, 0] = 0.0
        finished = torch.zeros(B, K, dtype=torch.bool, device=dev)
        lengths = torch.zeros(B, K, dtype=torch.int64, device=dev)
        tokens = torch.full((B * K,), self.start_token, dtype=torch.int64, device=dev)
        inputs = self.embedding_fn(_wrap(tokens)) if self.embedding_fn else _wrap(tokens)
        return inputs, (states, log_probs, finished, lengths), finished

    def step(self, time, inputs, states, **kwargs):
        cell_states, log_probs, finished, lengths = states
        B, K = log_probs.shape
        out, new_cell = self.cell(inputs, cell_states, **kwargs)
        logits = self.output_fn(out) if self.output_fn else out
        lp = torch.log_softmax(_unwrap(logits).float(), -1).reshape(B, K, -1)
        V = lp.shape[-1]
        eos_only = torch.full((V,), float('-inf'), device=lp.device)
        eos_only[self.end_token] = 0.0
        lp = torch.where(finished.unsqueeze(-1), eos_only, lp)
        scores = (log_probs.unsqueeze(-1) + lp).reshape(B, K * V)
        top, idx = scores.topk(K, -1)
        beam = idx // V
        tok = idx % V
        gather = (beam + torch.arange(B, device=lp.device).unsqueeze(1) * K).reshape(-1)
        new_cell = self._map(lambda s: _wrap(_unwrap(s)[gather]), new_cell)
        prev_fin = finished.gather(1, beam)
        new_fin = prev_fin | (tok == self.end_token)
        new_len = lengths.gather(1, beam) + (~prev_fin).long()
        nxt = self.embedding_fn(_wrap(tok.reshape(-1))) if self.embedding_fn else _wrap(tok.reshape(-1))
        outputs = (tok, beam)
        return outputs, (new_cell, top, new_fin, new_len), nxt, new_fin

    def finalize(self, outputs, final_states, sequence_lengths):
        toks = torch.stack([o[0] for o in outputs])  # [T, B, K]
        parents = torch.stack([o[1] for o in outputs])
        T = toks.shape[0]
        res = torch.empty_like(toks)
        par = torch.arange(toks.shape[2], device=toks.device).unsqueeze(0).expand_as(toks[0])
        for t in range(T - 1, -1, -1):
            res[t] = toks[t].gather(1, par)
            par = parents[t].gather(1, par)
        return _wrap(res), final_states


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False, impute_finished=False,
                   is_test=False, return_length=False, **kwargs):
    inputs, states, finished = decoder.initialize(inits)
    outputs = []
    step = 0
    while True:
        out, states, inputs, finished = decoder.step(step, inputs, states, **kwargs)
        outputs.append(out)
        step += 1
        if bool(finished.all()) or (max_step_num is not None and step > max_step_num):
            break
    final, final_states = decoder.finalize(outputs, states, None)
    t = _unwrap(final)
    if not output_time_major:
        t = t.permute(1, 2, 0) if t.dim() == 3 else t.transpose(0, 1)
    res = (_wrap(t), final_states)
    if return_length:
        res = res + (_wrap(states[3]),)
    return res
