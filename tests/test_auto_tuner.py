"""paddle.distributed.auto_tuner (reference python/paddle/distributed/auto_tuner/): candidate
generation, prune rules, the memory / step-time models, history-driven pruning, and the launcher's
--auto_tuner_json trial loop (CPU processes)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from paddle.distributed.auto_tuner import AutoTuner, estimate_memory_gb, estimate_step_time  # noqa: E402
from paddle.distributed.auto_tuner import prune as P  # noqa: E402

GPT13 = {'hidden_size': 2048, 'num_layers': 24, 'num_attention_heads': 16, 'vocab_size': 50304,
         'seq_length': 1024, 'global_batch_size': 128}
LLAMA13 = {'hidden_size': 5120, 'num_layers': 40, 'num_attention_heads': 40, 'vocab_size': 32000,
           'seq_length': 4096, 'global_batch_size': 64, 'intermediate_size': 13824 * 3 // 2}


def _cfg(**kw):
    c = dict(dp_degree=1, mp_degree=1, pp_degree=1, vpp_degree=1, sharding_degree=1, sharding_stage=None,
             micro_batch_size=1, use_recompute=False, recompute_granularity=None, acc_steps=1, num_gpus=8)
    c.update(kw)
    return c


def test_memory_model_orders_strategies():
    base = estimate_memory_gb(GPT13, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1))
    sh3 = estimate_memory_gb(GPT13, _cfg(sharding_degree=8, sharding_stage=3, micro_batch_size=16, acc_steps=1))
    rc = estimate_memory_gb(GPT13, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1, use_recompute=True,
                                        recompute_granularity='full'))
    assert sh3 < base and rc < base
    # the bench's GPT-3 1.3B at mb 16 fits one 288 GB MI355X (it runs there), 13B unsharded does not
    assert estimate_memory_gb(GPT13, _cfg(num_gpus=1, micro_batch_size=16)) < 288
    assert estimate_memory_gb(LLAMA13, _cfg(num_gpus=1, micro_batch_size=4)) > 288


def test_step_time_model_prefers_less_communication():
    t_dp = estimate_step_time(GPT13, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1), 8)
    t_mp = estimate_step_time(GPT13, _cfg(mp_degree=8, micro_batch_size=16, acc_steps=8), 8)
    t_pp = estimate_step_time(GPT13, _cfg(pp_degree=8, micro_batch_size=1, acc_steps=128), 8)
    assert t_dp < t_mp and t_dp < t_pp
    # more micro-batches shrink the bubble
    t_pp2 = estimate_step_time(GPT13, _cfg(pp_degree=8, micro_batch_size=1, acc_steps=16), 8)
    assert t_pp < t_pp2 * 8  # 8x the work in less than 8x the time


def test_prune_rules():
    tc = {'model_cfg': GPT13, 'gpus_per_node': 8, 'max_mem_usage': 288}
    assert 'mp' in P.prune(tc, _cfg(mp_degree=3, dp_degree=1, num_gpus=3))
    assert 'layers' in P.prune(tc, _cfg(pp_degree=5, num_gpus=5, acc_steps=8))
    assert 'acc' in P.prune(tc, _cfg(pp_degree=4, dp_degree=2, acc_steps=2))
    assert P.prune(tc, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1)) is None
    tiny = dict(tc, max_mem_usage=20)
    assert 'GB' in P.prune(tiny, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1))
    # history: micro batch 8 OOMed -> 16 pruned; no recompute fit -> recompute pruned
    hist = [dict(_cfg(dp_degree=8, micro_batch_size=8, acc_steps=2), oom=True, time=-1),
            dict(_cfg(dp_degree=8, micro_batch_size=4, acc_steps=4), oom=False, time=1.0)]
    assert 'memory' in P.prune(tc, _cfg(dp_degree=8, micro_batch_size=16, acc_steps=1), hist)
    assert 'lighter' in P.prune(tc, _cfg(dp_degree=8, micro_batch_size=4, acc_steps=4, use_recompute=True,
                                          recompute_granularity='full'), hist)


@pytest.mark.parametrize('algo', ['grid', 'cost_model'])
def test_tuner_loop_finds_the_best(algo):
    tc = {'model_cfg': GPT13, 'num_gpus': 8, 'gpus_per_node': 8, 'max_mem_usage': 288, 'task_limit': 400,
          'search_algo': {'name': algo}, 'metric_cfg': {'name': 'tokens_per_s', 'OptimizationDirection': 'Maximize'},
          'micro_batch_size': [1, 4, 16], 'vpp_degree': [1], 'recompute_granularity': ['full']}
    tuner = AutoTuner(tc)
    seen = []

    def fake_trial(cfg):  # the model's own prediction plays the measured throughput
        seen.append(cfg)
        t = estimate_step_time(GPT13, cfg, 8)
        return {'tokens_per_s': GPT13['global_batch_size'] * 1024 / t, 'oom': False}
    best = tuner.run(fake_trial)
    assert best is not None and len(seen) > 3
    keys = {tuple(sorted((k, v) for k, v in c.items() if k != 'job_id' and k != 'estimated_step_time'
                         and k != 'estimated_memory_usage')) for c in seen}
    assert len(keys) == len(seen)  # no candidate twice
    assert all(c['dp_degree'] * c['mp_degree'] * c['pp_degree'] * c['sharding_degree'] == 8 for c in seen)
    assert best['tokens_per_s'] == max(c['tokens_per_s'] for c in tuner.history_cfgs)
    if algo == 'cost_model':  # predicted-best first
        assert tuner.history_cfgs[0]['tokens_per_s'] == best['tokens_per_s']


def test_launch_auto_tuner_json_runs_trials(tmp_path):
    script = tmp_path / 'train.py'
    script.write_text(
        "import os, json, sys\n"
        "sys.path.insert(0, %r)\n"
        "from paddle.distributed.auto_tuner import current_trial\n"
        "c = current_trial()\n"
        "assert '--mbs' in sys.argv\n"
        "if int(os.environ['RANK']) == 0:\n"
        "    if c['micro_batch_size'] == 4: print('RuntimeError: HIP out of memory'); sys.exit(1)\n"
        "    print('ips: %%f' %% (100.0 * c['micro_batch_size'] / c['mp_degree']))\n" % ROOT)
    cfg = {'model_cfg': {'hidden_size': 64, 'num_layers': 4, 'num_attention_heads': 4, 'vocab_size': 128,
                         'seq_length': 32, 'global_batch_size': 8},
           'dp_degree': 'auto', 'mp_degree': 'auto', 'pp_degree': [1], 'vpp_degree': [1], 'sharding_degree': [1],
           'micro_batch_size': [1, 2, 4], 'use_recompute': [False],
           'metric_cfg': {'name': 'ips', 'OptimizationDirection': 'Maximize'},
           'run_cmd': {'micro_batch_size': ['--mbs', '{}']}}
    (tmp_path / 'tuner.json').write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, '-m', 'paddle.distributed.launch', '--nproc_per_node', '2',
                        '--log_dir', str(tmp_path / 'log'), '--auto_tuner_json', str(tmp_path / 'tuner.json'),
                        str(script)], env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    best = json.load(open(tmp_path / 'log' / 'best_cfg.json'))
    assert best['micro_batch_size'] == 2 and best['mp_degree'] == 1 and best['ips'] == 200.0
    hist = open(tmp_path / 'log' / 'history.csv').read()
    assert 'True' in hist  # the mbs 4 trial was recorded as out of memory
