"""Training callbacks (reference: python/paddle/hapi/callbacks.py — CallbackList:71, Callback:131,
ProgBarLogger:300, ModelCheckpoint:550, LRScheduler:619, EarlyStopping:719, VisualDL:883,
WandbCallback:999, ReduceLROnPlateau:1172)."""
import json
import numbers
import os
import sys
import time
import warnings

import numpy as np


def config_callbacks(callbacks=None, model=None, batch_size=None, epochs=None, steps=None, log_freq=2, verbose=2,
                     save_freq=1, save_dir=None, metrics=None, mode='train'):
    cbks = list(callbacks or [])
    if not any(isinstance(k, ProgBarLogger) for k in cbks) and verbose:
        cbks = [ProgBarLogger(log_freq, verbose=verbose)] + cbks
    if not any(isinstance(k, ModelCheckpoint) for k in cbks):
        cbks = cbks + [ModelCheckpoint(save_freq, save_dir)]
    if not any(isinstance(k, LRScheduler) for k in cbks):
        cbks = cbks + [LRScheduler()]
    cl = CallbackList(cbks)
    cl.set_model(model)
    metrics = metrics or [] if mode != 'test' else []
    cl.set_params({'batch_size': batch_size, 'epochs': epochs, 'steps': steps, 'verbose': verbose,
                   'metrics': metrics})
    return cl


class CallbackList:
    def __init__(self, callbacks=None):
        self.callbacks = list(callbacks or [])
        self.params = {}
        self.model = None

    def append(self, cb):
        self.callbacks.append(cb)

    def __iter__(self):
        return iter(self.callbacks)

    def set_params(self, params):
        self.params = params
        for c in self.callbacks:
            c.set_params(params)

    def set_model(self, model):
        self.model = model
        for c in self.callbacks:
            c.set_model(model)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def on_begin(self, mode, logs=None):
        self._call(f'on_{mode}_begin', logs)

    def on_end(self, mode, logs=None):
        self._call(f'on_{mode}_end', logs)

    def on_epoch_begin(self, epoch=None, logs=None):
        self._call('on_epoch_begin', epoch, logs)

    def on_epoch_end(self, epoch=None, logs=None):
        self._call('on_epoch_end', epoch, logs)

    def on_batch_begin(self, mode, step=None, logs=None):
        self._call(f'on_{mode}_batch_begin', step, logs)

    def on_batch_end(self, mode, step=None, logs=None):
        self._call(f'on_{mode}_batch_end', step, logs)


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_eval_begin(self, logs=None): pass
    def on_eval_end(self, logs=None): pass
    def on_predict_begin(self, logs=None): pass
    def on_predict_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, step, logs=None): pass
    def on_train_batch_end(self, step, logs=None): pass
    def on_eval_batch_begin(self, step, logs=None): pass
    def on_eval_batch_end(self, step, logs=None): pass
    def on_predict_batch_begin(self, step, logs=None): pass
    def on_predict_batch_end(self, step, logs=None): pass


def _fmt(logs, keys):
    out = []
    for k in keys:
        if k not in logs:
            continue
        v = logs[k]
        if isinstance(v, (list, tuple)) and len(v) == 1:
            v = v[0]
        if isinstance(v, numbers.Number):
            out.append(f"{k}: {v:.4f}" if isinstance(v, float) else f"{k}: {v}")
        elif isinstance(v, (list, tuple)):
            out.append(f"{k}: " + ' '.join(f"{x:.4f}" for x in v))
    return ' - '.join(out)


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq = log_freq
        self.verbose = verbose
        self._is_main = int(os.environ.get('RANK', '0')) == 0

    def _keys(self, logs):
        return [k for k in logs if k not in ('batch_size',)]

    def on_train_begin(self, logs=None):
        self.epochs = self.params.get('epochs')
        self.train_metrics = ['loss'] + list(self.params.get('metrics') or [])

    def on_epoch_begin(self, epoch=None, logs=None):
        self.epoch = epoch
        self.steps = self.params.get('steps')
        self._t0 = time.time()
        if self.verbose and self._is_main and self.epochs:
            print(f"Epoch {epoch + 1}/{self.epochs}", flush=True)

    def on_train_batch_end(self, step, logs=None):
        logs = logs or {}
        if self.verbose and self._is_main and (step + 1) % self.log_freq == 0:
            tot = f"/{self.steps}" if self.steps else ''
            print(f"step {step + 1}{tot} - {_fmt(logs, self._keys(logs))} - "
                  f"{(time.time() - self._t0) / (step + 1) * 1e3:.0f}ms/step", flush=True)

    def on_epoch_end(self, epoch, logs=None):
        if self.verbose == 1 and self._is_main:
            print(f"epoch {epoch + 1} - {_fmt(logs or {}, self._keys(logs or {}))}", flush=True)

    def on_eval_begin(self, logs=None):
        self._t0 = time.time()
        if self.verbose and self._is_main:
            print("Eval begin...", flush=True)

    def on_eval_end(self, logs=None):
        if self.verbose and self._is_main:
            print(f"Eval samples: {(logs or {}).get('batch_size', '')} - {_fmt(logs or {}, self._keys(logs or {}))}",
                  flush=True)

    def on_predict_begin(self, logs=None):
        if self.verbose and self._is_main:
            print("Predict begin...", flush=True)


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq = save_freq
        self.save_dir = save_dir

    def _main(self):
        return int(os.environ.get('RANK', '0')) == 0

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and self._main() and self.model is not None and (epoch + 1) % self.save_freq == 0:
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir and self._main() and self.model is not None:
            self.model.save(os.path.join(self.save_dir, 'final'))


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        if by_step and by_epoch:
            raise ValueError("by_step and by_epoch cannot both be True")
        self.by_step = by_step
        self.by_epoch = by_epoch

    def _sched(self):
        opt = getattr(self.model, '_optimizer', None)
        lr = getattr(opt, '_learning_rate', None) if opt is not None else None
        from ..optimizer.lr import LRScheduler as _S
        return lr if isinstance(lr, _S) else None

    def on_epoch_end(self, epoch, logs=None):
        s = self._sched()
        if self.by_epoch and s is not None:
            s.step()

    def on_train_batch_end(self, step, logs=None):
        s = self._sched()
        if self.by_step and s is not None:
            s.step()


class EarlyStopping(Callback):
    def __init__(self, monitor='loss', mode='auto', patience=0, verbose=1, min_delta=0, baseline=None,
                 save_best_model=True):
        super().__init__()
        self.monitor = monitor
        self.patience = patience
        self.verbose = verbose
        self.baseline = baseline
        self.min_delta = abs(min_delta)
        self.wait_epoch = 0
        self.best_weights = None
        self.stopped_epoch = 0
        self.save_best_model = save_best_model
        if mode not in ('auto', 'min', 'max'):
            warnings.warn(f"EarlyStopping mode {mode} is unknown, fallback to auto mode.")
            mode = 'auto'
        if mode == 'min' or (mode == 'auto' and 'acc' not in monitor):
            self.monitor_op, self.min_delta = np.less, -self.min_delta
        else:
            self.monitor_op = np.greater
        self.reset()

    def reset(self):
        self.wait_epoch = 0
        self.best_value = np.inf if self.monitor_op == np.less else -np.inf
        if self.baseline is not None:
            self.best_value = self.baseline

    def on_train_begin(self, logs=None):
        self.reset()

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            warnings.warn('Monitor of EarlyStopping should be loss or metric name.')
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        if self.monitor_op(cur - self.min_delta, self.best_value):
            self.best_value = cur
            self.wait_epoch = 0
            if self.save_best_model and self.params.get('save_dir'):
                self.model.save(os.path.join(self.params['save_dir'], 'best_model'))
        else:
            self.wait_epoch += 1
        if self.wait_epoch >= self.patience:
            self.model.stop_training = True
            if self.verbose > 0:
                print(f"Epoch {self.stopped_epoch + 1}: Early stopping.")
        self.stopped_epoch += 1


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor='loss', factor=0.1, patience=10, verbose=1, mode='auto', min_delta=1e-4, cooldown=0,
                 min_lr=0):
        super().__init__()
        if factor >= 1.0:
            raise ValueError('ReduceLROnPlateau does not support a factor >= 1.0.')
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.verbose, self.min_delta, self.cooldown, self.min_lr = verbose, min_delta, cooldown, min_lr
        self.mode = 'min' if (mode == 'min' or (mode == 'auto' and 'acc' not in monitor)) else 'max'
        self.cooldown_counter = 0
        self.wait = 0
        self.best = np.inf if self.mode == 'min' else -np.inf

    def _better(self, a, b):
        return a < b - self.min_delta if self.mode == 'min' else a > b + self.min_delta

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        opt = self.model._optimizer
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if self._better(cur, self.best):
            self.best = cur
            self.wait = 0
        elif self.cooldown_counter <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                old = float(opt.get_lr())
                if old > self.min_lr:
                    new = max(old * self.factor, self.min_lr)
                    opt.set_lr(new)
                    if self.verbose > 0:
                        print(f"ReduceLROnPlateau reducing learning rate to {new}.")
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


class VisualDL(Callback):
    """Scalar logging; VisualDL itself is not installed, so scalars go to ``log_dir/scalars.jsonl``."""

    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir
        self._step = 0

    def _write(self, tag, logs):
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, 'scalars.jsonl'), 'a') as f:
            for k, v in (logs or {}).items():
                v = v[0] if isinstance(v, (list, tuple)) and v else v
                if isinstance(v, numbers.Number):
                    f.write(json.dumps({'tag': f"{tag}/{k}", 'step': self._step, 'value': float(v)}) + '\n')

    def on_train_batch_end(self, step, logs=None):
        self._step += 1
        self._write('train', logs)

    def on_eval_end(self, logs=None):
        self._write('eval', logs)


class WandbCallback(Callback):
    def __init__(self, project=None, entity=None, name=None, dir=None, mode=None, job_type=None, **kwargs):  # noqa: A002
        super().__init__()
        warnings.warn("wandb is not installed (no network); WandbCallback records nothing", stacklevel=2)


_ = sys
