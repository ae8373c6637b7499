"""GEMM solution database for plain library GEMMs (hipBLASLt / rocBLAS via torch TunableOp).

Reference analogue: paddle.incubate.autotune (kernel autotune with a tuning range, results
cached per shape).  Here the per-shape winners for gfx950 are measured once on the box
(``tools/tune_gemms.sh``) and committed as ``configs/gemm_tuning_gfx950.csv``; every GPU
process loads them read-only on first device use, so the fresh-box bench pays no tuning time.
``autotune.set_config({'kernel': {'enable': True}})`` re-enables online tuning.
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DB = os.path.join(_HERE, 'configs', 'gemm_tuning_gfx950.csv')
_applied = [False]


def apply_tuned_db(path=None):
    """Enable TunableOp in read-only mode with the committed solution table (idempotent)."""
    if _applied[0] or not pa_flag('gemm_tuning'):
        return False
    path = path or DB
    if not os.path.exists(path):
        return False
    import torch
    if not torch.cuda.is_available():
        return False
    try:
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(False)
        t.set_filename(path)
        ok = t.read_file(path)
        t.write_file_on_exit(False) if hasattr(t, 'write_file_on_exit') else None
    except Exception:  # noqa: BLE001 - a stale table must never break training
        return False
    _applied[0] = True
    return ok


def enable_online_tuning(filename=None, max_duration_ms=30, max_iterations=100):
    import torch
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(True)
    t.set_max_tuning_duration(max_duration_ms)
    t.set_max_tuning_iterations(max_iterations)
    if filename:
        t.set_filename(filename)


def disable():
    import torch
    torch.cuda.tunable.enable(False)
