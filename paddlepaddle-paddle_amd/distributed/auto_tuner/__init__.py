"""paddle.distributed.auto_tuner — hybrid-parallel configuration search (reference:
python/paddle/distributed/auto_tuner/{tuner,search,prune,cost_model,memory_cost_model,recorder,utils}.py).

A tuner config (dict / JSON) names the model (``model_cfg``: hidden_size, num_layers,
num_attention_heads, vocab_size, seq_length, global_batch_size, intermediate_size), the machine
(``num_gpus``, ``nodes``, ``max_mem_usage`` in GB — 288 per MI355X by default), the search space
(``dp_degree`` / ``mp_degree`` / ``pp_degree`` / ``vpp_degree`` / ``sharding_degree`` /
``sharding_stage`` / ``micro_batch_size`` / ``use_recompute`` / ``recompute_granularity`` —
lists, or "auto" for every valid value) and the metric (``metric_cfg``: name, OptimizationDirection).

``AutoTuner.search_once()`` hands out the next candidate that survives the prune rules (shape
divisibility, GPU count, memory model, history: a config that OOMed prunes every config that needs
more memory); ``add_cfg`` records a trial's result; ``get_best`` / the recorder's CSV give the
ranking.  ``paddle.distributed.launch --auto_tuner_json cfg.json train.py ...`` runs the trials
(launch.auto_tune).  The ``cost_model`` search orders candidates by an analytic MI355X step-time
model (MFMA compute at a measured efficiency, tensor-parallel all-reduces and pipeline sends over
xGMI, the pipeline bubble, un-overlapped data-parallel / sharding collectives) so the first trials
are the likely winners.
"""
from .tuner import AutoTuner  # noqa: F401
from .recorder import HistoryRecorder  # noqa: F401
from .memory_cost_model import estimate_memory_gb  # noqa: F401
from .cost_model import estimate_step_time  # noqa: F401
from .utils import default_candidates, search_all  # noqa: F401



def current_trial():
    """The candidate config of the auto-tuner trial this process belongs to (None outside one)."""
    import json
    import os
    v = os.environ.get('PADDLE_AUTO_TUNER_CFG')
    return json.loads(v) if v else None


__all__ = []
