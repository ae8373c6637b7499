"""Post-training quantisation of static inference models (reference:
python/paddle/static/quantization/post_training_quantization.py PostTrainingQuantization /
PostTrainingQuantizationProgram / WeightQuantization).

Flow: load the fp32 inference model (reference ProgramDesc, PIR json or this framework's IR) →
observe the activation input of every quantisable op over the calibration batches through the
Executor (abs-max / per-batch abs-max / histogram, csrc-free torch reductions on the device) →
thresholds by ``algo`` → each quantised GEMM becomes one int8 node (``paddle.ops.int8.quant_linear``:
int8 weights with per-channel scales, per-tensor activation threshold, the int8 MFMA GEMM on the
GPU), each conv a fixed quant-dequant conv → ``save_quantized_model`` writes an inference model the
Predictor / ``load_inference_model`` run as is.
"""
import copy
import os

import numpy as np
import torch

from ..program import Node, Ref
from . import calibration as C
from .passes import find_sites, freeze_site, DEFAULT_TYPES, weight_scales, _const_tensor, _add_const

_OBS = {'on': None, 'phase': 'range'}


def observe(x, key=None):
    """Calibration probe node: records statistics of ``x`` under ``key``, returns x."""
    reg = _OBS['on']
    if reg is not None and isinstance(x, torch.Tensor):
        o = reg.setdefault(key, C.Observer())
        if _OBS['phase'] == 'range':
            o.observe_range(x)
        else:
            o.observe_hist(x)
    return x


class PostTrainingQuantizationProgram:
    def __init__(self, executor, program, feed_list=None, fetch_list=None, scope=None, batch_generator=None,
                 sample_generator=None, data_loader=None, batch_size=10, batch_nums=None, algo="KL",
                 hist_percent=0.99999, quantizable_op_type=("conv2d", "depthwise_conv2d", "mul"), round_type='round',
                 learning_rate=0.001, is_full_quantize=False, bias_correction=False, activation_bits=8,
                 weight_bits=8, activation_quantize_type='range_abs_max',
                 weight_quantize_type='channel_wise_abs_max', onnx_format=False, freeze_model=True,
                 optimize_model=False, is_use_cache_file=False, skip_tensor_list=None, same_scale_tensor_list=None,
                 cache_dir=None, scale_dict=None, return_graph=True, **kw):
        if algo not in ('KL', 'hist', 'avg', 'mse', 'emd', 'abs_max', 'min_max', 'ptf'):
            raise ValueError(f"unsupported algo {algo}")
        if weight_quantize_type not in ('abs_max', 'channel_wise_abs_max'):
            raise ValueError(f"unsupported weight_quantize_type {weight_quantize_type}")
        if sum(x is not None for x in (batch_generator, sample_generator, data_loader)) != 1:
            raise ValueError("exactly one of sample_generator, batch_generator and data_loader must be set")
        self._exe = executor
        self._program = program
        self._feed_list = list(feed_list or [])
        self._fetch_list = list(fetch_list or [])
        self._batch_generator, self._sample_generator, self._data_loader = batch_generator, sample_generator, data_loader
        self._batch_size, self._batch_nums = batch_size, batch_nums
        self._algo = 'abs_max' if algo == 'ptf' else algo
        self._hist_percent = hist_percent
        self._types = tuple(quantizable_op_type) if quantizable_op_type else DEFAULT_TYPES
        self._abits, self._wbits = activation_bits, weight_bits
        self._channel_wise = weight_quantize_type == 'channel_wise_abs_max'
        self._freeze = freeze_model
        self._skip = set(skip_tensor_list or [])
        self._scale_dict = dict(scale_dict or {})
        self._return_graph = return_graph
        self._quantized = None
        self._scales = {}

    # ---- data
    def _feeds(self, names):
        n = 0
        if self._data_loader is not None:
            it = self._data_loader() if callable(self._data_loader) else self._data_loader
            for batch in it:
                yield self._as_feed(batch, names)
                n += 1
                if self._batch_nums and n >= self._batch_nums:
                    return
            return
        if self._batch_generator is not None:
            for batch in self._batch_generator():
                yield self._as_feed(batch, names)
                n += 1
                if self._batch_nums and n >= self._batch_nums:
                    return
            return
        buf = []
        for sample in self._sample_generator():
            buf.append(sample if isinstance(sample, (list, tuple)) else (sample,))
            if len(buf) == self._batch_size:
                yield self._as_feed([np.stack([np.asarray(s[i]) for s in buf]) for i in range(len(buf[0]))], names)
                buf = []
                n += 1
                if self._batch_nums and n >= self._batch_nums:
                    return

    @staticmethod
    def _as_feed(batch, names):
        if isinstance(batch, dict):
            return batch
        if not isinstance(batch, (list, tuple)):
            batch = [batch]
        return {nm: (b._t if hasattr(b, '_t') else b) for nm, b in zip(names, batch)}

    def _feed_names(self):
        if self._feed_list:
            return [f if isinstance(f, str) else f.name for f in self._feed_list]
        return list(self._program.feeds.keys())

    def _fetch(self):
        if self._fetch_list:
            return self._fetch_list
        return list(getattr(self._program, '_fetch_vars', []))[:1]

    # ---- calibration
    def _probe_program(self, sites):
        p = copy.copy(self._program)
        nodes = list(self._program.nodes)
        out = []
        keys = {}
        for s in sites:
            keys[s.idx] = f"act_{s.act.vid}"
            s.key = keys[s.idx]
        for i, n in enumerate(nodes):
            if i in keys:
                s = next(x for x in sites if x.idx == i)
                out.append(Node('torch', observe, [Ref(s.act.vid)], {'key': keys[i]}, s.act.vid))
            out.append(n)
        p.nodes = out
        p._ir_cache = None
        p._ir_optim = False  # calibrate the ops as recorded
        return p

    def _run(self, prog, names, phase):
        _OBS['phase'] = phase
        for feed in self._feeds(names):
            self._exe.run(prog, feed=feed, fetch_list=self._fetch())

    def quantize(self):
        prog = self._program
        sites = [s for s in find_sites(prog, self._types)]
        names = self._feed_names()
        probe = self._probe_program(sites)
        reg = {}
        _OBS['on'] = reg
        try:
            from ..program import _paused  # noqa: F401
            import paddle
            was_static = paddle.in_dynamic_mode() is False
            paddle.enable_static()
            try:
                self._run(probe, names, 'range')
                if C.needs_hist(self._algo):
                    for o in reg.values():
                        o.hist_max = o.absmax
                    self._run(probe, names, 'hist')
            finally:
                if not was_static:
                    paddle.disable_static()
        finally:
            _OBS['on'] = None
        for s in sites:
            o = reg.get(s.key)
            if s.key in self._scale_dict:
                self._scales[s.key] = float(self._scale_dict[s.key])
            elif o is not None:
                self._scales[s.key] = C.threshold(o, self._algo, self._abits, self._hist_percent)
        # the quantised program (in place: the reference returns the rewritten graph)
        nodes = list(prog.nodes)
        for s in sites:
            sc = self._scales.get(s.key)
            if sc is None or s.key in self._skip:
                continue
            n = nodes[s.idx]
            if self._freeze:
                nodes[s.idx] = freeze_site(prog, n, s.weight, s.act, s.layout, sc, self._wbits, self._abits,
                                           self._channel_wise)
            else:
                nodes[s.idx] = _fake_quant_site(prog, n, s, sc, self._wbits, self._abits, self._channel_wise)
        flat = []
        for n in nodes:
            if isinstance(n, _Seq):
                flat.extend(n)
            else:
                flat.append(n)
        prog.nodes[:] = flat
        prog._ir_cache = None
        prog._quant_scales = dict(self._scales)
        self._quantized = prog
        return prog

    def save_quantized_model(self, save_model_path, model_filename=None, params_filename=None):
        from ..io import save_inference_model
        prog = self._quantized if self._quantized is not None else self._program
        prefix = save_model_path
        if os.path.isdir(save_model_path) or model_filename is not None or save_model_path.endswith(os.sep):
            base = (model_filename or 'model.pdmodel').replace('.pdmodel', '')
            prefix = os.path.join(save_model_path, base)
        feeds = [prog.named_vars[n] for n in self._feed_names() if n in prog.named_vars]
        save_inference_model(prefix, feeds, self._fetch() or list(getattr(prog, '_fetch_vars', [])), self._exe,
                             program=prog)
        return prefix


def _fake_quant_site(prog, n, s, act_scale, wbits, abits, channel_wise):
    """freeze_model=False: fixed activation quant-dequant + quant-dequantised weight, float op."""
    from ...ops.int8 import fake_quant_dequant
    w = _const_tensor(prog, s.weight)
    q, ws = weight_scales(w, s.layout, wbits, channel_wise)
    qmax = 2 ** (wbits - 1) - 1
    if s.layout == 'conv':
        wd = q.float() * (ws / qmax).reshape(-1, *([1] * (q.dim() - 1)))
    else:
        wd = q.float() * (ws / qmax)[:, None]
        if s.layout == 'kn':
            wd = wd.t()
    wc = _add_const(prog, wd.to(w.dtype).contiguous())
    v = next(prog._vid)
    pre = Node('torch', fake_quant_dequant, [s.act], {'scale': float(act_scale), 'bits': abits}, v)
    args = [Ref(v) if (isinstance(a, Ref) and a.vid == s.act.vid) else
            (wc if (hasattr(a, 'cid') and a.cid == s.weight.cid) else a) for a in n.args]
    node = Node(n.kind, n.target, args, dict(n.kwargs), n.outs, dict(n.meta or {}, quantized='fake'))
    return _Seq([pre, node])


class _Seq(list):
    pass


class PostTrainingQuantization(PostTrainingQuantizationProgram):
    """PTQ of a saved inference model (``model_dir`` + model / params file names)."""

    def __init__(self, executor, model_dir, scope=None, model_filename=None, params_filename=None,
                 batch_generator=None, sample_generator=None, data_loader=None, batch_size=10, batch_nums=None,
                 algo="KL", hist_percent=0.99999, quantizable_op_type=[], round_type='round',  # noqa: B006
                 learning_rate=0.001, is_full_quantize=False, bias_correction=False, activation_bits=8,
                 weight_bits=8, activation_quantize_type='range_abs_max',
                 weight_quantize_type='channel_wise_abs_max', onnx_format=False, freeze_model=True,
                 optimize_model=False, is_use_cache_file=False, skip_tensor_list=None, same_scale_tensor_list=None,
                 cache_dir=None, scale_dict=None, return_graph=False, deploy_backend=None):
        from ..io import load_inference_model
        prefix = model_dir
        if model_filename is not None:
            prefix = os.path.join(model_dir, model_filename.rsplit('.pdmodel', 1)[0])
        elif os.path.isdir(model_dir):
            cands = [f for f in os.listdir(model_dir) if f.endswith('.pdmodel') or f.endswith('.json')]
            if not cands:
                raise ValueError(f"no inference model in {model_dir}")
            prefix = os.path.join(model_dir, cands[0].rsplit('.', 1)[0])
        prog, feed_names, fetch = load_inference_model(prefix, executor)
        super().__init__(executor, prog, feed_names, fetch, scope, batch_generator, sample_generator, data_loader,
                         batch_size, batch_nums, algo, hist_percent, quantizable_op_type or DEFAULT_TYPES,
                         round_type, learning_rate, is_full_quantize, bias_correction, activation_bits, weight_bits,
                         activation_quantize_type, weight_quantize_type, onnx_format, freeze_model, optimize_model,
                         is_use_cache_file, skip_tensor_list, same_scale_tensor_list, cache_dir, scale_dict,
                         return_graph)


class WeightQuantization:
    """Weight-only quantisation of a saved inference model (reference WeightQuantization):
    ``quantize_weight_to_int`` stores the quantisable GEMM weights as int8 / int16 values with
    per-channel (or per-tensor) scales and runs them on the weight-only path."""

    def __init__(self, model_dir, model_filename=None, params_filename=None):
        self._model_dir, self._model_filename = model_dir, model_filename

    def quantize_weight_to_int(self, save_model_dir, save_model_filename=None, save_params_filename=None,
                               quantizable_op_type=("conv2d", "mul"), weight_bits=8, weight_quantize_type="channel_wise_abs_max",
                               generate_test_model=False, threshold_rate=0.0):
        import paddle
        from ..io import load_inference_model, save_inference_model
        from .passes import QuantWeightPass
        exe = paddle.static.Executor(paddle.CPUPlace())
        prefix = self._model_dir if self._model_filename is None else os.path.join(
            self._model_dir, self._model_filename.rsplit('.pdmodel', 1)[0])
        if os.path.isdir(prefix):
            cands = [f for f in os.listdir(prefix) if f.endswith('.pdmodel')]
            prefix = os.path.join(prefix, cands[0].rsplit('.', 1)[0])
        prog, feeds, fetch = load_inference_model(prefix, exe)
        QuantWeightPass(quant_bits=weight_bits).apply(prog)
        out = os.path.join(save_model_dir, (save_model_filename or 'model.pdmodel').rsplit('.pdmodel', 1)[0])
        save_inference_model(out, [prog.named_vars[f] for f in feeds], fetch, exe, program=prog)
        return out

    def convert_weight_to_fp16(self, save_model_dir):
        raise NotImplementedError("use paddle.inference.convert_to_mixed_precision for fp16 / bf16 weights")
