"""Collective watchdog (reference: paddle/fluid/distributed/collective/comm_task_manager.cc,
FLAGS_enable_async_trace / comm timeout reporting).

Every collective issued through ``paddle.distributed`` registers a task (op, group ranks,
shape/dtype, issue time, Python stack).  A daemon thread polls outstanding async works; a
task older than ``timeout_s`` is reported once with everything needed to find the rank that
did not arrive (and, with ``abort=True``, the process exits so the launcher tears the job
down instead of hanging).  Enabled by ``PADDLE_COMM_WATCHDOG=1`` or ``enable(timeout_s)``.
"""
import os
import sys
import threading
import time
import traceback

_lock = threading.Lock()
_tasks = {}
_next = [0]
_state = {'enabled': os.environ.get('PADDLE_COMM_WATCHDOG', '0') == '1',
          'timeout': float(os.environ.get('PADDLE_COMM_TIMEOUT_S', '600')), 'abort': False, 'thread': None,
          'reports': []}


def enable(timeout_s=600.0, abort=False):
    _state.update(enabled=True, timeout=float(timeout_s), abort=abort)
    _start()


def disable():
    _state['enabled'] = False


def enabled():
    return _state['enabled']


def _start():
    if _state['thread'] is None:
        th = threading.Thread(target=_loop, name='paddle-comm-watchdog', daemon=True)
        th.start()
        _state['thread'] = th


def begin(op, group_ranks, tensor=None, work=None):
    if not _state['enabled']:
        return None
    _start()
    desc = ''
    if tensor is not None and hasattr(tensor, 'shape'):
        desc = f"{tuple(tensor.shape)} {str(getattr(tensor, 'dtype', ''))}"
    with _lock:
        tid = _next[0]
        _next[0] += 1
        _tasks[tid] = {'op': op, 'ranks': group_ranks, 'desc': desc, 't0': time.time(), 'work': work,
                       'stack': ''.join(traceback.format_stack(limit=8)[:-2]), 'reported': False}
    return tid


def attach(tid, work):
    if tid is None:
        return
    with _lock:
        if tid in _tasks:
            _tasks[tid]['work'] = work


def end(tid):
    if tid is None:
        return
    with _lock:
        _tasks.pop(tid, None)


def pending():
    with _lock:
        return [dict(t, id=k) for k, t in _tasks.items()]


def reports():
    return list(_state['reports'])


def _loop():
    while True:
        time.sleep(min(1.0, max(_state['timeout'] / 10, 0.05)))
        if not _state['enabled']:
            continue
        now = time.time()
        done = []
        with _lock:
            items = list(_tasks.items())
        for tid, t in items:
            w = t['work']
            if w is not None:
                try:
                    if w.is_completed():
                        done.append(tid)
                        continue
                except Exception:  # noqa: BLE001
                    pass
            if not t['reported'] and now - t['t0'] > _state['timeout']:
                t['reported'] = True
                rank = os.environ.get('RANK', '0')
                msg = (f"[paddle comm watchdog] rank {rank}: {t['op']} {t['desc']} on ranks {t['ranks']} "
                       f"pending for {now - t['t0']:.1f}s (timeout {_state['timeout']}s); issued at:\n{t['stack']}")
                _state['reports'].append(msg)
                print(msg, file=sys.stderr, flush=True)
                if _state['abort']:
                    os._exit(6)
        if done:
            with _lock:
                for tid in done:
                    _tasks.pop(tid, None)
