"""Multi-process (gloo, world_size 2) tests of the distributed engines on CPU."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def run_workers(script, *args, nproc=2, timeout=300):
    env = dict(os.environ)
    env['CUDA_VISIBLE_DEVICES'] = ''
    env['HIP_VISIBLE_DEVICES'] = ''
    env['PYTHONPATH'] = ROOT
    env['OMP_NUM_THREADS'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr=127.0.0.1', f'--master-port={_port()}', os.path.join(ROOT, 'tests', 'dist', script), *args]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


@pytest.mark.parametrize("mode", ['dp', 'os', 'os_g', 'p_g_os', 'p_g_os_keep', 'os_g_offload', 'p_g_os_offload'])
def test_dp_and_sharding_match_single_process(mode):
    out = run_workers('worker_dp_sharding.py', mode)
    assert out.count(f'{mode} OK') == 2


def test_tensor_parallel_with_data_parallel_syncs_gradients():
    out = run_workers('worker_hybrid.py', 'tpdp', nproc=4)
    assert out.count('tpdp OK') == 4, out[-3000:]


@pytest.mark.parametrize("kind", ['momentum', 'sgd'])
@pytest.mark.parametrize("mode", ['os', 'p_g_os', 'p_g_os_offload'])
def test_sharded_momentum_sgd_match_single_process(mode, kind):
    out = run_workers('worker_dp_sharding.py', mode, kind)
    assert out.count(f'{mode} OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['tp', 'sp', 'pp', 'vpp'])
def test_hybrid_parallel_matches_single_device(mode):
    out = run_workers('worker_hybrid.py', mode)
    assert out.count(f'{mode} OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['os', 'os_g', 'p_g_os'])
def test_gpt_sharding_matches_single_process(mode):
    out = run_workers('worker_gpt_sharding.py', mode)
    assert out.count(f"gpt {mode} OK") == 2, out[-3000:]


def test_gpt_sharding_fp32_reduce_scatter():
    """fp32 main-grad communication: bf16/fp32 gradients reduce-scattered in fp32 into an fp32 arena."""
    out = run_workers('worker_gpt_sharding.py', 'p_g_os', 'float32')
    assert out.count("gpt p_g_os-float32 OK") == 2, out[-3000:]


def test_auto_parallel_reshard_and_dist_checkpoint(tmp_path):
    os.environ['CKPT_DIR'] = str(tmp_path / 'ckpt')
    out = run_workers('worker_auto_parallel.py')
    assert out.count("auto_parallel OK") == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['plain', 'stage1', 'stage2', 'distmodel'])
def test_auto_parallel_shard_optimizer_matches_single_process(mode):
    out = run_workers('worker_auto_shard.py', mode)
    assert out.count(f"auto_shard {mode} OK") == 2, out[-3000:]


def test_comm_watchdog_reports_stuck_collective():
    out = run_workers('worker_watchdog.py', timeout=120)
    assert out.count("watchdog OK") == 2, out[-3000:]


def test_launch_module_spawns_workers(tmp_path):
    script = tmp_path / 'w.py'
    script.write_text("import os\nprint('worker', os.environ['RANK'], os.environ['PADDLE_TRAINERS_NUM'], "
                      "os.environ['FLAGS_selected_gpus'], flush=True)\n")
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, '-m', 'paddle.distributed.launch', '--devices', '0,1', '--log_dir',
                        str(tmp_path / 'log'), str(script)], env=env, capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'worker 0 2 0' in r.stdout
    assert 'worker 1 2 1' in (tmp_path / 'log' / 'workerlog.1').read_text()


@pytest.mark.parametrize("kind", ['linear', 'ffn'])
def test_moe_expert_parallel_matches_single_process(kind):
    out = run_workers('worker_moe.py', kind)
    assert out.count("moe OK") == 2, out[-3000:]


def test_rpc_sync_async_between_workers():
    out = run_workers('worker_rpc.py', str(_port()), timeout=180)
    assert out.count("rpc OK") == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['pp', 'vpp', 'vpp8'])
def test_pipeline_four_stages(mode):
    """4 ranks: 1F1B, the interleaved forward-then-backward (accumulate 4 = pp) and the interleaved
    1F1B (accumulate 8 = 2 pp) virtual-stage schedules match single-device SGD."""
    out = run_workers('worker_hybrid.py', mode, nproc=4)
    assert out.count(f'{mode} OK') == 4, out[-3000:]


def test_auto_parallel_spmd_propagation_matches_single_process():
    out = run_workers('worker_spmd.py', timeout=180)
    assert out.count("spmd OK") == 2, out[-3000:]


def test_parameter_server_sync_sgd_matches_full_batch():
    """2 parameter servers + 2 trainers (dense slices + sharded sparse embedding table)."""
    servers = [f"127.0.0.1:{_port()}" for _ in range(2)]
    base = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='1', CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='',
                PADDLE_PSERVERS_IP_PORT_LIST=','.join(servers), PADDLE_TRAINERS_NUM='2',
                PADDLE_PS_MASTER_ENDPOINT=f"127.0.0.1:{_port()}")
    procs = []
    for role, idx in (('PSERVER', 0), ('PSERVER', 1), ('TRAINER', 0), ('TRAINER', 1)):
        env = dict(base, TRAINING_ROLE=role)
        env['PADDLE_PSERVER_ID' if role == 'PSERVER' else 'PADDLE_TRAINER_ID'] = str(idx)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, 'tests', 'dist', 'worker_ps.py')], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    text = '\n'.join(outs)
    assert all(p.returncode == 0 for p in procs), text[-4000:]
    assert text.count('ps OK') == 4, text[-3000:]


def test_launch_elastic_restart_and_ps_mode(tmp_path):
    """--max_restart relaunches a failed job (workers see the restart count); --run_mode ps spawns
    servers + trainers with the PS environment."""
    script = tmp_path / 'flaky.py'
    script.write_text("import os, sys\nc = int(os.environ['PADDLE_ELASTIC_RESTART_COUNT'])\n"
                      "print('attempt', c, os.environ['RANK'], flush=True)\nsys.exit(3 if c == 0 else 0)\n")
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable, '-m', 'paddle.distributed.launch', '--nproc_per_node', '2', '--max_restart', '2',
                        '--log_dir', str(tmp_path / 'log'), str(script)], env=env, capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'attempt 0 0' in r.stdout and 'attempt 1 0' in r.stdout and 'elastic restart 1/2' in r.stderr
    ps = tmp_path / 'ps.py'
    ps.write_text("import os\nprint(os.environ['TRAINING_ROLE'], os.environ.get('PADDLE_PSERVER_ID', os.environ.get("
                  "'PADDLE_TRAINER_ID')), os.environ['PADDLE_PSERVERS_IP_PORT_LIST'].count(','), flush=True)\n")
    r = subprocess.run([sys.executable, '-m', 'paddle.distributed.launch', '--run_mode', 'ps', '--server_num', '2',
                        '--trainer_num', '2', '--log_dir', str(tmp_path / 'pslog'), str(ps)], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert 'TRAINER 0 1' in r.stdout
    assert 'PSERVER 1 1' in (tmp_path / 'pslog' / 'serverlog.1').read_text()


def test_llama_hybrid_tp2_pp2_matches_single_device():
    out = run_workers('worker_llama_hybrid.py', nproc=4, timeout=300)
    assert out.count('llama hybrid OK') == 4, out[-4000:]


def test_elastic_scale_out_and_in(tmp_path):
    """Elastic collective job (reference fleet/elastic ElasticManager, np=MIN:MAX): 2 nodes start a
    world of 2; a third node joining re-launches everyone with world 3 (scale out); killing it
    re-launches the survivors with world 2 (scale in); workers see the restart count."""
    import json
    import signal
    import time
    import datetime
    from torch.distributed import TCPStore
    port = _port()
    store = TCPStore('127.0.0.1', port, is_master=True, wait_for_workers=False,
                     timeout=datetime.timedelta(seconds=30))
    out = tmp_path / 'out'
    out.mkdir()
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', OMP_NUM_THREADS='1')

    def node(name):
        cmd = [sys.executable, '-m', 'paddle.distributed.launch', '--elastic_server', f'127.0.0.1:{port}',
               '--np', '2:3', '--job_id', 'ej', '--host', name, '--elastic_ttl', '3', '--log_dir',
               str(tmp_path / name), os.path.join(ROOT, 'tests', 'dist', 'worker_elastic.py'), str(out)]
        return subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                start_new_session=True)

    def worlds(timeout, want_world, nranks):
        t_end = time.time() + timeout
        while time.time() < t_end:
            gens = {}
            for f in out.glob('gen*_rank*'):
                g, r = f.name[3:].split('_rank')
                txt = f.read_text().split()
                if len(txt) == 3:
                    gens.setdefault(int(g), {})[int(r)] = tuple(map(int, txt))
            for g in sorted(gens, reverse=True):
                if len(gens[g]) == nranks and all(v[0] == want_world and v[1] == want_world
                                                   for v in gens[g].values()):
                    return g, gens[g]
            time.sleep(0.2)
        raise AssertionError(f"no generation with world {want_world}: {sorted(p.name for p in out.iterdir())}")

    procs = {n: node(n) for n in ('nodeA', 'nodeB')}
    try:
        g1, _ = worlds(90, 2, 2)
        procs['nodeC'] = node('nodeC')
        g2, r2 = worlds(90, 3, 3)
        assert g2 > g1 and max(v[2] for v in r2.values()) >= 1  # relaunched workers see the restart count
        os.killpg(procs['nodeC'].pid, signal.SIGKILL)  # node failure
        procs['nodeC'].wait()
        t_end = time.time() + 90
        while True:
            g3, _ = worlds(max(1, t_end - time.time()), 2, 2)
            if g3 > g2:
                break
        (out / 'stop').write_text('1')
        for n in ('nodeA', 'nodeB'):
            rc = procs[n].wait(timeout=60)
            log = procs[n].stdout.read().decode(errors='replace')
            assert rc == 0, log[-3000:]
        assert json.loads(store.get('ej/members').decode()) == []
        assert store.get('ej/done').decode() == '1'
    finally:
        for p in procs.values():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass


@pytest.mark.parametrize("clip", ['0', '0.5'])
def test_llama_hybrid_tp2_pp2_sharding2_matches_single_device(clip):
    """The fleet sharding axis (8 gloo ranks): sharded AdamW state, reduce-scattered gradients,
    global-norm clipping across sharding x mp x pp, equal to single-device training."""
    os.environ['CLIP'] = clip
    try:
        out = run_workers('worker_llama_hybrid_sharding.py', nproc=8, timeout=600)
    finally:
        os.environ.pop('CLIP', None)
    assert out.count("sharding2 OK") == 8, out[-3000:]


def test_distributed_scaler_agrees_on_overflow():
    out = run_workers('worker_scaler.py')
    assert out.count('scaler OK') == 2, out[-3000:]


@pytest.mark.parametrize("clip,shard", [('0', '1'), ('0.05', '1'), ('0.05', '0')])
def test_pipeline_shared_weight_with_sharding(clip, shard):
    """SharedLayerDesc (tied embedding / head across two stages) with sharding_degree 2 (or a
    plain dp axis): the shared weight's gradient is summed over the stages; clipping counts it once."""
    os.environ['CLIP'], os.environ['SHARD'] = clip, shard
    try:
        out = run_workers('worker_pp_shared_sharding.py', nproc=4, timeout=300)
    finally:
        os.environ.pop('CLIP', None)
        os.environ.pop('SHARD', None)
    assert out.count("shared-weight OK") == 4, out[-3000:]


def test_fused_multi_transformer_ring_id_tensor_parallel():
    out = run_workers('worker_fmt_tp.py', nproc=2, timeout=300)
    assert out.count("fmt tp OK") == 2, out[-3000:]


@pytest.mark.parametrize("nproc", [2, 4])
def test_bench_multi_rank_path_rehearsal(nproc):
    """bench.py's N-rank flow (one process per device, sharding-3 GPT + data-parallel ResNet,
    barrier-bracketed timing, MAX over ranks, one JSON line from rank 0) on gloo with tiny models."""
    import json
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', PYTHONPATH=ROOT, OMP_NUM_THREADS='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={nproc}',
           '--master-addr=127.0.0.1', f'--master-port={_port()}', os.path.join(ROOT, 'bench.py'), '--cpu',
           '--model', 'gpt-tiny', '--steps', '2', '--warmup', '1', '--resnet-model', 'resnet18', '--resnet-batch', '2',
           '--micro-batch', '2', '--seq', '64', '--gpus', str(nproc)]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d['n_gpus'] == nproc and d['config']['parallelism'] == f'sharding-3x{nproc}'
    assert d['config']['global_batch'] == 2 * nproc and d['resnet50']['config']['parallelism'] == f'dp{nproc}'
    assert d['value'] > 0 and abs(d['value'] - 2 * 64 * nproc / (d['ms_per_step'] / 1e3)) < 1e-2 * d['value']


def test_bench_gpus_flag_launches_its_own_ranks():
    """``python bench.py --gpus 2`` with no launcher starts the 2 ranks itself (no HIP call in the
    parent) and reports the collective world size; a launcher / --gpus mismatch is an error."""
    import json
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', PYTHONPATH=ROOT, OMP_NUM_THREADS='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    args = ['--cpu', '--model', 'gpt-tiny', '--steps', '2', '--warmup', '1', '--resnet-model', 'resnet18',
            '--resnet-batch', '2', '--micro-batch', '2', '--seq', '64']
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args, '--gpus', '2'], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['world_size'] == 2 and d['config']['parallelism'] == 'sharding-3x2'
    assert d['backend'] == 'gloo'
    # the timed steps trained on different batches: a finite, non-memorised loss
    assert 0.5 < d['final_loss'] < 20
    bad = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
                          '--master-addr=127.0.0.1', f'--master-port={_port()}', os.path.join(ROOT, 'bench.py'),
                          *args, '--gpus', '4'], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         timeout=600)
    assert bad.returncode != 0 and 'launcher started 2' in bad.stderr


@pytest.mark.parametrize("mode", ['fleet', 'fleet_merge', 'pass'])
def test_static_collective_data_parallel_matches_full_batch(mode):
    out = run_workers('worker_static_dp.py', mode)
    assert out.count(f'static dp {mode} OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode,nproc", [('tp', 2), ('tpdp', 4)])
def test_static_fleet_tensor_parallel(mode, nproc):
    """Static-mode fleet with mpu layers: collectives recorded as program nodes; shards match a
    single-process full-weight run."""
    out = run_workers('worker_static_tp.py', mode, nproc=nproc)
    assert out.count(f'static {mode} OK') == nproc, out[-3000:]


@pytest.mark.parametrize("sched,mode,nproc", [('1F1B', 'pp', 2), ('FThenB', 'pp', 2), ('1F1B', 'pp', 3),
                                              ('1F1B', 'ppdp', 4), ('1F1B', 'ppamp', 2), ('FThenB', 'ppgm', 2),
                                              ('ZBH1', 'pp', 2), ('ZBH1', 'pp', 3), ('ZBH1', 'ppdp', 4),
                                              ('VPP', 'pp', 2), ('VPP', 'pp', 4), ('VPP', 'ppdp', 4)])
def test_static_fleet_pipeline_parallel(sched, mode, nproc):
    """Static-mode fleet pipeline: device_guard stages, micro-batched FThenB / 1F1B with
    send/recv of activations and gradients; every stage's parameters match a single-process run."""
    out = run_workers('worker_static_pp.py', sched, mode, nproc=nproc)
    assert out.count(f'static pp {sched} {mode} OK') == nproc, out[-3000:]


@pytest.mark.parametrize('k', [1, 2])
def test_dist_to_static_program_data_parallel(k):
    """dist.to_static records the step into a static Program; batch-sharded inputs on 2 ranks
    give the single-process full-batch result (gradient merge k = 2 too)."""
    out = run_workers('worker_dist_static.py', str(k))
    assert out.count(f'dist static k{k} OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode", ['shard1', 'shard2', 'shard3', 'pp_1F1B', 'pp_FThenB', 'pp_ZBH1', 'engine'])
def test_dist_to_static_sharded_and_pipelined_programs(mode):
    """dist.to_static / auto.Engine with sharding stage 1/2/3 or a 2-stage pipeline run as static
    Programs and equal single-process training (tests/dist/worker_dist_static_sp.py)."""
    out = run_workers('worker_dist_static_sp.py', mode)
    assert out.count(f'dist static {mode} OK') == 2, out[-3000:]


def test_dist_to_static_tensor_parallel_program():
    """dist.to_static with column / row-parallel placements records the SPMD-propagated step
    (per-shard ops + reshard collectives as program nodes) and equals single-process training."""
    out = run_workers('worker_dist_static_tp.py')
    assert out.count('dist static tp OK') == 2, out[-3000:]


def test_dist_to_static_full_auto_planner():
    """strategy.auto_mode = 'full': the rule-based planner finds the attention and FFN blocks of a
    transformer layer and places them column / row parallel; the static step equals one process."""
    out = run_workers('worker_dist_auto_plan.py')
    assert out.count('dist auto plan OK') == 2, out[-3000:]


@pytest.mark.parametrize("mode,nproc", [('sep', 2), ('sepmp', 4), ('sepdp', 4), ('sepsh', 4)])
def test_segment_parallel_matches_single_process(mode, nproc):
    """sep alone and x mp / dp / sharding: gradients summed over sep, averaged over dp
    (reference fleet/utils/hybrid_parallel_util.py:241), weights broadcast over sep."""
    out = run_workers('worker_sep.py', mode, nproc=nproc)
    assert out.count(f'{mode} OK') == nproc, out[-3000:]


@pytest.mark.parametrize("mode,nproc", [('zbh1', 2), ('zbh1_8', 4)])
def test_zero_bubble_pipeline_matches_single_device(mode, nproc):
    """ZB-H1 (backward split into B and deferred W, dX sent before W) trains exactly like the
    single-device model (reference passes/pipeline_scheduler_pass/pipeline_zero_bubble.py)."""
    out = run_workers('worker_hybrid.py', mode, nproc=nproc)
    assert out.count(f'{mode} OK') == nproc, out[-3000:]


def test_zero_bubble_schedule_shrinks_the_bubble():
    """The schedule shape: every stage's op list played against the others (unit F / B / W costs):
    ZB-H1's bubble is (S-1)(F+B) against 1F1B's (S-1)(F+B+W)."""
    sys.path.insert(0, ROOT)
    from paddle.distributed.fleet.meta_parallel.zero_bubble_utils import simulate, schedule_order
    for S, M in [(2, 4), (4, 8), (8, 16), (8, 32)]:
        m1, b1 = simulate('1F1B', S, M)
        mz, bz = simulate('ZBH1', S, M)
        assert m1 == 3 * M + 3 * (S - 1) and mz == 3 * M + 2 * (S - 1), (S, M, m1, mz)
        assert bz < b1
        for s in range(S):  # every micro-batch's F, B and W exactly once per stage
            ops = schedule_order('ZBH1', S, s, M)
            assert sorted(ops) == sorted([(k, i) for k in 'FBW' for i in range(M)])
