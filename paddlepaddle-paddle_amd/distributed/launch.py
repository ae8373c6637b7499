"""``python -m paddle.distributed.launch`` (reference: python/paddle/distributed/launch/main.py,
controllers/collective.py).

Collective mode (one process per MI355X): spawns ``--nproc_per_node`` (or one per entry of
``--devices/--gpus``) workers with the env the reference sets (PADDLE_TRAINER_ID,
PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ENDPOINTS, FLAGS_selected_gpus) plus torch.distributed's
(RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT), pins each worker to its GPU through
``HIP_VISIBLE_DEVICES``-free LOCAL_RANK selection, writes ``<log_dir>/workerlog.<i>``, and
tears every worker down if one fails (exit code of the first failure is returned).

Elastic restart (reference launch ``--max_restart`` / fleet elastic fault tolerance): with
``--max_restart N`` a failed job is torn down and relaunched (fresh rendezvous port) up to N
times; workers see ``PADDLE_ELASTIC_RESTART_COUNT`` and resume from their checkpoints.

Elastic scale in / out (reference fleet/elastic/manager.py, launch ``--elastic_server``/``--np``):
with ``--elastic_server host:port --np MIN:MAX`` each launcher is one node of an elastic job
(distributed/elastic.py, a TCPStore registry with heartbeats): it waits until MIN..MAX nodes
are alive, launches its workers with that generation's ranks/world, and when nodes join or
disappear tears its workers down and re-rendezvouses with the new world
(``PADDLE_ELASTIC_GEN`` / ``PADDLE_ELASTIC_RESTART_COUNT`` tell workers to resume from their
checkpoints).  A worker failure is retried up to ``--max_restart`` times.

Parameter-server mode (``--run_mode ps`` with ``--server_num``/``--trainer_num``, reference
controllers/ps.py): servers and trainers get TRAINING_ROLE, PADDLE_PSERVERS_IP_PORT_LIST,
PADDLE_PSERVER_ID / PADDLE_TRAINER_ID, PADDLE_TRAINERS_NUM (see distributed/ps).
"""
import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def parse_args(argv=None):
    ap = argparse.ArgumentParser('paddle.distributed.launch')
    ap.add_argument('--master', default=None, help='ip:port of the rank-0 node')
    ap.add_argument('--rank', type=int, default=0, help='node rank')
    ap.add_argument('--nnodes', type=str, default='1')
    ap.add_argument('--nproc_per_node', type=int, default=None)
    ap.add_argument('--devices', '--gpus', dest='devices', default=None)
    ap.add_argument('--log_dir', default='log')
    ap.add_argument('--job_id', default='default')
    ap.add_argument('--run_mode', default='collective')
    ap.add_argument('--max_restart', type=int, default=0)
    ap.add_argument('--server_num', type=int, default=None)
    ap.add_argument('--trainer_num', type=int, default=None)
    ap.add_argument('--elastic_server', default=None, help='host:port of the elastic TCPStore')
    ap.add_argument('--np', default=None, help='elastic node count: N or MIN:MAX')
    ap.add_argument('--host', default=None, help='this node\'s name in the elastic registry')
    ap.add_argument('--elastic_ttl', type=float, default=6.0)
    ap.add_argument('--elastic_timeout', type=float, default=600.0)
    ap.add_argument('--auto_tuner_json', default=None,
                    help='search hybrid-parallel configs (distributed/auto_tuner): one trial job per candidate')
    ap.add_argument('training_script')
    ap.add_argument('training_script_args', nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _wait(procs):
    """Wait for all; on the first failure stop the rest.  Returns the first non-zero code."""
    rc = 0
    alive = list(procs)
    while alive:
        for p, log in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove((p, log))
            if r != 0 and rc == 0:
                rc = r
                for q, _ in alive:  # one worker failed: stop the job
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.2)
    return rc


def _spawn(cmd, env, log_path, to_console):
    log = open(log_path, 'w')
    p = subprocess.Popen(cmd, env=env, stdout=None if to_console else log,
                         stderr=None if to_console else subprocess.STDOUT, start_new_session=True)
    return p, log


def _collective(a, attempt, restart_count=None):
    devices = a.devices.split(',') if a.devices else None
    nproc = a.nproc_per_node or (len(devices) if devices else 1)
    devices = devices or [str(i) for i in range(nproc)]
    nnodes = int(str(a.nnodes).split(':')[0])
    if a.master:
        host, port = a.master.rsplit(':', 1)
        port = str(int(port) + attempt) if attempt else port
    else:
        host, port = '127.0.0.1', str(_free_port())
    world = nnodes * nproc
    endpoints = ','.join(f"{host}:{int(port) + i}" for i in range(world))
    procs = []
    for i in range(nproc):
        rank = a.rank * nproc + i
        env = dict(os.environ)
        env.update({'RANK': str(rank), 'LOCAL_RANK': str(i), 'WORLD_SIZE': str(world), 'LOCAL_WORLD_SIZE': str(nproc),
                    'MASTER_ADDR': host, 'MASTER_PORT': port, 'PADDLE_TRAINER_ID': str(rank),
                    'PADDLE_TRAINERS_NUM': str(world), 'PADDLE_TRAINER_ENDPOINTS': endpoints,
                    'PADDLE_CURRENT_ENDPOINT': f"{host}:{int(port) + rank}", 'FLAGS_selected_gpus': devices[i],
                    'PADDLE_JOB_ID': a.job_id, 'PADDLE_LOCAL_DEVICE_IDS': devices[i],
                    'PADDLE_ELASTIC_RESTART_COUNT': str(attempt if restart_count is None else restart_count)})
        cmd = [sys.executable, '-u', a.training_script] + a.training_script_args
        procs.append(_spawn(cmd, env, os.path.join(a.log_dir, f"workerlog.{i}"),
                            i == 0 and not getattr(a, 'log_all', False)))
    return procs


def _kill(procs):
    for p, _ in procs:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    for p, _ in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass


def _elastic(a):
    """One node of an elastic collective job (see module docstring)."""
    from .elastic import ElasticManager, connect_store
    node = a.host or f"{socket.gethostname()}-{os.getpid()}"
    store = connect_store(a.elastic_server)
    mgr = ElasticManager(store, a.job_id, node, a.np or a.nnodes, ttl=a.elastic_ttl)
    mgr.register()
    restarts = 0
    try:
        while True:
            if mgr.completed():
                return 0
            gen, members = mgr.wait_for_np(timeout=a.elastic_timeout)
            nrank, nnodes = mgr.rank(), len(members)
            if nrank == 0:
                mgr.publish_master(f"127.0.0.1:{_free_port()}")
            master = mgr.wait_master()
            print(f"[launch] elastic generation {gen}: node {node} rank {nrank}/{nnodes} master {master}",
                  file=sys.stderr, flush=True)
            a2 = argparse.Namespace(**vars(a))
            a2.master, a2.rank, a2.nnodes = master, nrank, str(nnodes)
            os.environ['PADDLE_ELASTIC_GEN'] = str(gen)
            procs = _collective(a2, 0, restart_count=restarts)
            try:
                while True:
                    codes = [p.poll() for p, _ in procs]
                    if all(c == 0 for c in codes):
                        mgr.exit(completed=True)
                        return 0
                    if any(c not in (None, 0) for c in codes):
                        rc = next(c for c in codes if c not in (None, 0))
                        if mgr.completed():
                            return rc
                        if restarts >= a.max_restart and not mgr.changed():
                            mgr.exit()
                            return rc
                        break  # fault tolerance: re-rendezvous (peers see the same failure)
                    if not mgr.completed() and mgr.changed():
                        print(f"[launch] elastic membership changed (generation {gen}); relaunching",
                              file=sys.stderr, flush=True)
                        break
                    time.sleep(0.25)
            finally:
                _kill(procs)
                for _, log in procs:
                    log.close()
            restarts += 1
    except KeyboardInterrupt:
        return 130
    finally:
        mgr._stop.set()


def _ps(a, attempt):
    ns, nt = a.server_num or 1, a.trainer_num or 1
    servers = [f"127.0.0.1:{_free_port()}" for _ in range(ns)]
    base = dict(os.environ, PADDLE_PSERVERS_IP_PORT_LIST=','.join(servers), PADDLE_TRAINERS_NUM=str(nt),
                PADDLE_PS_MASTER_ENDPOINT=f"127.0.0.1:{_free_port()}", PADDLE_JOB_ID=a.job_id,
                PADDLE_ELASTIC_RESTART_COUNT=str(attempt))
    cmd = [sys.executable, '-u', a.training_script] + a.training_script_args
    procs = []
    for i in range(ns):
        env = dict(base, TRAINING_ROLE='PSERVER', PADDLE_PSERVER_ID=str(i), PADDLE_PORT=servers[i].split(':')[1])
        procs.append(_spawn(cmd, env, os.path.join(a.log_dir, f"serverlog.{i}"), False))
    for i in range(nt):
        env = dict(base, TRAINING_ROLE='TRAINER', PADDLE_TRAINER_ID=str(i))
        procs.append(_spawn(cmd, env, os.path.join(a.log_dir, f"workerlog.{i}"), i == 0))
    return procs


def auto_tune(a):
    """--auto_tuner_json: run the training script once per candidate of the auto tuner
    (reference launch/main.py auto-tuner mode).  Each trial gets the candidate as JSON in
    PADDLE_AUTO_TUNER_CFG (``paddle.distributed.auto_tuner.current_trial()``) and, per the tuner
    config's ``run_cmd`` ({key: [flag, template]}), as script arguments; the metric is parsed from
    worker 0's log (``metric_cfg.name: value``), an out-of-memory failure is recorded as such.
    The history CSV and the best config land in ``log_dir``."""
    import json
    import re
    from .auto_tuner import AutoTuner
    with open(a.auto_tuner_json) as f:
        tcfg = json.load(f)
    tcfg.setdefault('num_gpus', a.nproc_per_node or len((a.devices or '0').split(',')))
    tcfg.setdefault('gpus_per_node', tcfg['num_gpus'])
    tuner = AutoTuner(tcfg)
    metric = tuner.recorder.metric
    pat = re.compile(re.escape(metric) + r"\s*[:=]\s*([-+0-9.eE]+)")
    base_args = list(a.training_script_args)

    def trial(cfg):
        d = os.path.join(a.log_dir, f"trial{cfg['job_id']}")
        os.makedirs(d, exist_ok=True)
        a2 = argparse.Namespace(**vars(a))
        a2.log_dir = d
        a2.log_all = True  # worker 0 to its log too: the metric is read from there
        a2.nproc_per_node = cfg['num_gpus']
        args = list(base_args)
        for k, (flag, tmpl) in (tcfg.get('run_cmd') or {}).items():
            if cfg.get(k) is not None:
                args += [flag, str(tmpl).format(cfg[k])]
        a2.training_script_args = args
        os.environ['PADDLE_AUTO_TUNER_CFG'] = json.dumps(cfg)
        try:
            procs = _collective(a2, 0)
            try:
                rc = _wait(procs)
            finally:
                for _, log in procs:
                    log.close()
        finally:
            os.environ.pop('PADDLE_AUTO_TUNER_CFG', None)
        text = ''
        for fn in sorted(os.listdir(d)):
            with open(os.path.join(d, fn), errors='replace') as f:
                text += f.read()
        oom = 'out of memory' in text.lower() or 'outofmemory' in text.lower()
        vals = pat.findall(text)
        if rc != 0 or not vals:
            return {metric: -1, 'oom': oom}
        return {metric: float(vals[-1]), 'oom': False}
    best = tuner.run(trial, history_csv_path=os.path.join(a.log_dir, 'history.csv'))
    with open(os.path.join(a.log_dir, 'best_cfg.json'), 'w') as f:
        json.dump(best, f)
    print(f"[launch] auto tuner best config: {best}", file=sys.stderr, flush=True)
    return 0 if best is not None else 1


def launch(argv=None):
    a = parse_args(argv)
    if a.auto_tuner_json:
        os.makedirs(a.log_dir, exist_ok=True)
        return auto_tune(a)
    if a.run_mode not in ('collective', 'ps'):
        raise SystemExit(f"unsupported run_mode {a.run_mode!r} (collective | ps)")
    os.makedirs(a.log_dir, exist_ok=True)
    if a.elastic_server:
        if a.run_mode != 'collective':
            raise SystemExit("elastic scaling is supported for collective jobs")
        return _elastic(a)
    rc = 0
    for attempt in range(a.max_restart + 1):
        procs = (_ps if a.run_mode == 'ps' else _collective)(a, attempt)
        try:
            rc = _wait(procs)
        except KeyboardInterrupt:
            for p, _ in procs:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
            return 130
        finally:
            for _, log in procs:
                log.close()
        if rc == 0:
            return 0
        if attempt < a.max_restart:
            print(f"[launch] job failed with exit code {rc}; elastic restart {attempt + 1}/{a.max_restart}",
                  file=sys.stderr, flush=True)
    return rc


def main():
    sys.exit(launch())


if __name__ == '__main__':
    main()
