"""``python -m paddle.distributed.launch`` (reference: python/paddle/distributed/launch/main.py,
controllers/collective.py).

Collective mode only (one process per MI355X): spawns ``--nproc_per_node`` (or one per entry of
``--devices/--gpus``) workers with the env the reference sets (PADDLE_TRAINER_ID,
PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ENDPOINTS, FLAGS_selected_gpus) plus torch.distributed's
(RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT), pins each worker to its GPU through
``HIP_VISIBLE_DEVICES``-free LOCAL_RANK selection, writes ``<log_dir>/workerlog.<i>``, and
tears every worker down if one fails (exit code of the first failure is returned).
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
    ap.add_argument('training_script')
    ap.add_argument('training_script_args', nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def launch(argv=None):
    a = parse_args(argv)
    if a.run_mode != 'collective':
        raise SystemExit("only collective mode is supported (parameter-server mode is out of scope)")
    devices = a.devices.split(',') if a.devices else None
    nproc = a.nproc_per_node or (len(devices) if devices else 1)
    devices = devices or [str(i) for i in range(nproc)]
    nnodes = int(str(a.nnodes).split(':')[0])
    if a.master:
        host, port = a.master.rsplit(':', 1)
    else:
        host, port = '127.0.0.1', str(_free_port())
    world = nnodes * nproc
    os.makedirs(a.log_dir, exist_ok=True)
    endpoints = ','.join(f"{host}:{int(port) + i}" for i in range(world))
    procs = []
    for i in range(nproc):
        rank = a.rank * nproc + i
        env = dict(os.environ)
        env.update({'RANK': str(rank), 'LOCAL_RANK': str(i), 'WORLD_SIZE': str(world), 'LOCAL_WORLD_SIZE': str(nproc),
                    'MASTER_ADDR': host, 'MASTER_PORT': port, 'PADDLE_TRAINER_ID': str(rank),
                    'PADDLE_TRAINERS_NUM': str(world), 'PADDLE_TRAINER_ENDPOINTS': endpoints,
                    'PADDLE_CURRENT_ENDPOINT': f"{host}:{int(port) + rank}", 'FLAGS_selected_gpus': devices[i],
                    'PADDLE_JOB_ID': a.job_id, 'PADDLE_LOCAL_DEVICE_IDS': devices[i]})
        log = open(os.path.join(a.log_dir, f"workerlog.{i}"), 'w')
        cmd = [sys.executable, '-u', a.training_script] + a.training_script_args
        p = subprocess.Popen(cmd, env=env, stdout=log if i else None, stderr=subprocess.STDOUT if i else None,
                             start_new_session=True)
        procs.append((p, log))
    rc = 0
    try:
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
    except KeyboardInterrupt:
        for p, _ in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        rc = 130
    finally:
        for _, log in procs:
            log.close()
    return rc


def main():
    sys.exit(launch())


if __name__ == '__main__':
    main()
