"""paddle.incubate.autotune (reference: python/paddle/incubate/autotune.py set_config).

``kernel``: GEMM solution tuning (hipBLASLt/rocBLAS via TunableOp) — enabled online tuning
measures every candidate for each new shape within ``tuning_range`` steps, then freezes.
``layout``: channels-last preference for conv nets (NHWC feeds MIOpen's fast path).
``dataloader``: picks ``num_workers`` automatically when a DataLoader is created with -1.
"""
import json

_config = {'kernel': {'enable': False, 'tuning_range': [1, 10]}, 'layout': {'enable': False},
           'dataloader': {'enable': False, 'tuning_steps': 500}}


def set_config(config=None):
    if config is None:
        config = {'kernel': {'enable': True}, 'layout': {'enable': True}, 'dataloader': {'enable': True}}
    if isinstance(config, str):
        with open(config) as f:
            config = json.load(f)
    for k, v in config.items():
        if k in _config:
            _config[k].update(v)
    if _config['kernel']['enable']:
        try:
            from ..ops.gemm_tuning import enable_online_tuning
            enable_online_tuning()
        except Exception:  # noqa: BLE001 - no GPU
            pass


def get_config():
    return {k: dict(v) for k, v in _config.items()}
