"""Elastic membership for collective jobs: scale in / scale out / fault tolerance.

Reference: python/paddle/distributed/fleet/elastic/manager.py (``ElasticManager``: etcd-backed
node registry with leased heartbeats, ``np = "MIN:MAX"``, ``_update_elastic_scale_out`` /
``_update_elastic_scale_in`` re-ranking that keeps surviving nodes in place, ``ElasticStatus``
HOLD / RESTART / COMPLETED / EXIT) and launch/controllers/master.py (peer sync).

Design here: no etcd in this stack, so the coordination service is a ``torch.distributed``
``TCPStore`` (the same key-value service the collectives rendezvous on).  State per job:

* ``{job}/members``  JSON list of node names in JOIN order (ranks = list positions, so a
  scale-in closes the gap without moving the nodes before it and a scale-out appends);
  modified only by compare-and-set, together with ``{job}/gen`` (bumped on every change).
* ``{job}/hb/{node}`` last heartbeat (wall clock) — written by a daemon thread per node; a node
  whose heartbeat is older than ``ttl`` is pruned by whichever peer notices first.
* ``{job}/gen{g}/master`` the rendezvous endpoint chosen by generation ``g``'s rank-0 node.
* ``{job}/done`` set once a node's workers finished successfully (no relaunch after that).

The launcher (``distributed/launch.py --elastic_server``) runs one ElasticManager per node:
``wait_for_np`` blocks until MIN <= live nodes <= MAX and the view is stable for ``settle``
seconds, workers are spawned with that generation's world, and ``changed`` (polled while
they run) tells the launcher to tear them down and re-rendezvous when nodes join or leave.
"""
import json
import os
import threading
import time


class ElasticStatus:
    COMPLETED = 'completed'
    ERROR = 'error'
    HOLD = 'hold'
    RESTART = 'restart'
    EXIT = 'exit'


class ElasticLevel:
    FAULT_TOLERANCE = 1
    ELASTIC = 2


def parse_np(np_str):
    """'N' or 'MIN:MAX' (reference ElasticManager._parse_np)."""
    s = str(np_str or os.environ.get('PADDLE_ELASTIC_NP', '1'))
    parts = s.split(':')
    lo = max(int(parts[0]), 1)
    hi = int(parts[1]) if len(parts) > 1 else lo
    return lo, max(hi, lo)


def connect_store(server, is_master=False, timeout=60.0):
    import datetime
    from torch.distributed import TCPStore
    host, port = server.rsplit(':', 1)
    return TCPStore(host, int(port), is_master=is_master, timeout=datetime.timedelta(seconds=timeout),
                    wait_for_workers=False)


class ElasticManager:
    def __init__(self, store, job_id, node, np='1', ttl=6.0, heartbeat=1.0, settle=2.0):
        self.store = store
        self.job = job_id
        self.node = node
        self.min_np, self.max_np = parse_np(np)
        self.ttl = ttl
        self.hb_interval = heartbeat
        self.settle = settle
        self.elastic_level = ElasticLevel.ELASTIC if self.max_np > self.min_np else ElasticLevel.FAULT_TOLERANCE
        self._stop = threading.Event()
        self._hb = None
        self.gen = None
        self.members = []

    # ---- store helpers
    def _k(self, *parts):
        return '/'.join([self.job] + [str(p) for p in parts])

    def _get(self, key, default=None):
        if self.store.check([key]):
            return self.store.get(key).decode()
        return default

    def _members(self):
        return json.loads(self._get(self._k('members'), '[]'))

    def _update_members(self, fn):
        """CAS loop: members <- fn(members); bumps the generation when the list changes."""
        key = self._k('members')
        while True:
            raw = self._get(key, None)
            cur = json.loads(raw) if raw is not None else []
            new = fn(list(cur))
            if new == cur:
                return cur
            expected = raw if raw is not None else ''
            got = self.store.compare_set(key, expected, json.dumps(new)).decode()
            if got == json.dumps(new):
                self.store.add(self._k('gen'), 1)
                return new

    def generation(self):
        return self.store.add(self._k('gen'), 0)

    # ---- membership
    def register(self):
        self.store.set(self._k('hb', self.node), repr(time.time()))
        self._update_members(lambda m: m if self.node in m else m + [self.node])
        if self._hb is None:
            self._hb = threading.Thread(target=self._heartbeat, daemon=True)
            self._hb.start()

    def _heartbeat(self):
        while not self._stop.wait(self.hb_interval):
            try:
                self.store.set(self._k('hb', self.node), repr(time.time()))
            except Exception:  # store gone: the job is over
                return

    def alive(self):
        """Members with a fresh heartbeat; stale ones are pruned from the registry."""
        now = time.time()
        members = self._members()
        dead = []
        for n in members:
            hb = self._get(self._k('hb', n))
            if hb is None or now - float(hb) > self.ttl:
                dead.append(n)
        if dead and self.node not in dead:
            members = self._update_members(lambda m: [n for n in m if n not in dead])
        return [n for n in members if n not in dead]

    def completed(self):
        return self._get(self._k('done')) == '1'

    def mark_completed(self):
        self.store.set(self._k('done'), '1')

    def wait_for_np(self, timeout=600.0, poll=0.25):
        """Blocks until MIN <= live nodes <= MAX and the view is stable for `settle` s.
        Returns (generation, members) for this node to launch with (HOLD while waiting)."""
        t_end = time.time() + timeout
        stable_since, last = None, None
        while time.time() < t_end:
            if self.node not in self._members():
                self.register()  # pruned while partitioned / slow: re-join at the end
            live = self.alive()
            view = (self.generation(), tuple(live))
            if view != last:
                last, stable_since = view, time.time()
            ok = self.min_np <= len(live) <= self.max_np and self.node in live
            if ok and time.time() - stable_since >= self.settle:
                self.gen, self.members = view[0], list(live)
                return self.gen, self.members
            time.sleep(poll)
        raise TimeoutError(f"elastic job {self.job}: {len(last[1]) if last else 0} live nodes, "
                           f"need {self.min_np}..{self.max_np}")

    def changed(self):
        """True when the live membership differs from the generation this node launched."""
        live = self.alive()
        return self.generation() != self.gen or live != self.members

    def rank(self):
        return self.members.index(self.node)

    def publish_master(self, endpoint):
        self.store.set(self._k(f'gen{self.gen}', 'master'), endpoint)

    def wait_master(self, timeout=60.0):
        key = self._k(f'gen{self.gen}', 'master')
        t_end = time.time() + timeout
        while time.time() < t_end:
            v = self._get(key)
            if v:
                return v
            time.sleep(0.1)
        raise TimeoutError(f"no rendezvous endpoint for generation {self.gen}")

    def exit(self, completed=False):
        self._stop.set()
        if completed:
            self.mark_completed()
        try:
            self._update_members(lambda m: [n for n in m if n != self.node])
        except Exception:
            pass
