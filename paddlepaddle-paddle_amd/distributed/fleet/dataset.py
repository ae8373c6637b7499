"""Slot-file datasets for the static Executor (reference: python/paddle/distributed/fleet/dataset/
dataset.py — DatasetBase / InMemoryDataset / QueueDataset / FileInstantDataset; executor.py
train_from_dataset / infer_from_dataset) and sparse-table entry configs (entry_attr.py).

Input files are piped through ``pipe_command`` (any shell command, default ``cat``; typically a
``fleet.MultiSlotDataGenerator`` script) and parsed as MultiSlot text: per instance, for every
variable of ``use_var`` in order, ``<n> v1 ... vn``.  A variable with ``lod_level == 0`` must carry
the same number of values in every instance (its feed is [batch, n]); a ``lod_level == 1`` variable
is variable-length and is fed as a LoD tensor (values concatenated, sequence lengths attached).
The reader threads of the reference are Python threads over files here (``thread_num``);
InMemoryDataset keeps parsed instances in host memory, shuffles locally or globally (an all-to-all
of instances over the trainers' gloo/RCCL group) and releases them; QueueDataset streams.
"""
import random
import shlex
import subprocess
import threading

import numpy as np


class _Entry:
    _name = ''

    def _to_attr(self):
        raise NotImplementedError


class ProbabilityEntry(_Entry):
    """Admit a new sparse feature with probability ``probability``."""

    def __init__(self, probability):
        if not isinstance(probability, float) or not 0 < probability <= 1:
            raise ValueError("probability must be a float in (0, 1]")
        self._name, self._probability = 'probability_entry', probability

    def _to_attr(self):
        return ":".join([self._name, str(self._probability)])


class CountFilterEntry(_Entry):
    """Admit a sparse feature once it has been seen ``count_filter`` times."""

    def __init__(self, count_filter):
        if not isinstance(count_filter, int) or count_filter < 0:
            raise ValueError("count_filter must be a non-negative int")
        self._name, self._count_filter = 'count_filter_entry', count_filter

    def _to_attr(self):
        return ":".join([self._name, str(self._count_filter)])


class ShowClickEntry(_Entry):
    """Sparse-feature admission driven by show / click statistics slots."""

    def __init__(self, show_name, click_name):
        if not isinstance(show_name, str) or not isinstance(click_name, str):
            raise ValueError("show_name and click_name must be str")
        self._name, self._show_name, self._click_name = 'show_click_entry', show_name, click_name

    def _to_attr(self):
        return ":".join([self._name, self._show_name, self._click_name])


def _var_meta(v):
    from ...static.program import static_shape
    name = getattr(v, 'name', None)
    lod = int(v.__dict__.get('_lod_level', getattr(v, 'lod_level', 0)) or 0) if hasattr(v, '__dict__') \
        else int(getattr(v, 'lod_level', 0) or 0)
    try:
        dtype = str(v.dtype).replace('paddle.', '').replace('torch.', '')
    except Exception:
        dtype = 'int64'
    shape = static_shape(v) if hasattr(v, '_t') else list(getattr(v, 'shape', []))
    return name, lod, dtype, shape


class DatasetBase:
    def __init__(self):
        self.batch_size = 1
        self.thread_num = 1
        self.use_var = []
        self.pipe_command = 'cat'
        self.input_type = 0
        self.filelist = []
        self.download_cmd = 'cat'
        self.fs_name = self.fs_ugi = ''

    def init(self, batch_size=1, thread_num=1, use_var=None, pipe_command="cat", input_type=0, fs_name="",
             fs_ugi="", download_cmd="cat", **kwargs):
        self._set_batch_size(batch_size)
        self._set_thread(thread_num)
        self._set_use_var(use_var or [])
        self._set_pipe_command(pipe_command)
        self.input_type = input_type
        self.fs_name, self.fs_ugi, self.download_cmd = fs_name, fs_ugi, download_cmd

    def _set_batch_size(self, n):
        self.batch_size = int(n)

    def _set_thread(self, n):
        self.thread_num = max(1, int(n))

    def _set_pipe_command(self, cmd):
        self.pipe_command = cmd

    def _set_use_var(self, var_list):
        self.use_var = list(var_list)
        self._metas = [_var_meta(v) for v in self.use_var]

    def set_filelist(self, filelist):
        self.filelist = list(filelist)

    # ---- parsing
    def _read_file(self, path):
        """Instances of one file: list of per-variable value lists."""
        cmd = self.pipe_command.strip()
        if cmd in ('', 'cat'):
            with open(path) as f:
                text = f.read()
        else:
            with open(path) as f:
                r = subprocess.run(shlex.split(cmd) if not any(c in cmd for c in '|;&<>') else cmd,
                                   stdin=f, capture_output=True, text=True, shell=any(c in cmd for c in '|;&<>'))
            if r.returncode != 0:
                raise RuntimeError(f"pipe_command '{cmd}' failed on {path}: {r.stderr.strip()}")
            text = r.stdout
        out = []
        nv = len(self._metas)
        for ln, line in enumerate(text.splitlines()):
            toks = line.split()
            if not toks:
                continue
            inst, i = [], 0
            for vi in range(nv):
                if i >= len(toks):
                    raise ValueError(f"{path}:{ln + 1}: {nv} slots expected, line ends after {vi}")
                n = int(toks[i])
                vals = toks[i + 1:i + 1 + n]
                if len(vals) != n:
                    raise ValueError(f"{path}:{ln + 1}: slot {vi} declares {n} values, {len(vals)} present")
                inst.append(vals)
                i += 1 + n
            if i != len(toks):
                raise ValueError(f"{path}:{ln + 1}: {len(toks) - i} trailing tokens after {nv} slots")
            out.append(inst)
        return out

    def _read_files(self, files):
        if self.thread_num <= 1 or len(files) <= 1:
            res = []
            for f in files:
                res.extend(self._read_file(f))
            return res
        parts = [None] * len(files)
        sem = threading.Semaphore(self.thread_num)
        errs = []

        def work(i, f):
            with sem:
                try:
                    parts[i] = self._read_file(f)
                except Exception as e:  # surfaced after join
                    errs.append(e)
        ts = [threading.Thread(target=work, args=(i, f)) for i, f in enumerate(files)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return [x for p in parts for x in p]

    # ---- batching
    def _batch_feed(self, insts):
        import paddle
        feed = {}
        for vi, (name, lod, dtype, shape) in enumerate(self._metas):
            np_dt = np.float32 if 'float' in dtype else np.int64
            cols = [np.asarray(inst[vi], dtype=np_dt) for inst in insts]
            if lod == 0:
                lens = {len(c) for c in cols}
                if len(lens) != 1:
                    raise ValueError(f"variable {name} (lod_level 0) got instances of lengths {sorted(lens)}")
                arr = np.stack(cols)
                tail = [s for s in shape[1:]]
                if tail and all(s > 0 for s in tail) and int(np.prod(tail)) == arr.shape[1]:
                    arr = arr.reshape([len(insts)] + tail)
                feed[name] = arr
            else:
                flat = np.concatenate(cols).reshape(-1, 1) if cols else np.zeros((0, 1), np_dt)
                t = paddle.to_tensor(flat)
                t.set_recursive_sequence_lengths([[len(c) for c in cols]])
                feed[name] = t
        return feed

    def _batches(self, insts):
        bs = self.batch_size
        for i in range(0, len(insts), bs):
            yield self._batch_feed(insts[i:i + bs])

    def _iter_batches(self):
        raise NotImplementedError


class InMemoryDataset(DatasetBase):
    def __init__(self):
        super().__init__()
        self._data = []
        self._loaded = False
        self._fleet_send_batch_size = 1024
        self.queue_num = None
        self.merge_by_lineid = False
        self.parse_ins_id = self.parse_content = False

    def init(self, **kwargs):
        base = {k: kwargs.pop(k) for k in ('batch_size', 'thread_num', 'use_var', 'pipe_command', 'input_type',
                                             'fs_name', 'fs_ugi', 'download_cmd') if k in kwargs}
        super().init(**base)
        self.update_settings(**kwargs)

    def update_settings(self, **kwargs):
        for k, v in kwargs.items():
            if k in ('batch_size', 'thread_num', 'use_var', 'pipe_command'):
                getattr(self, f'_set_{"thread" if k == "thread_num" else k}')(v)
            else:
                setattr(self, k, v)

    def _set_queue_num(self, n):
        self.queue_num = n

    def _set_parse_ins_id(self, v):
        self.parse_ins_id = bool(v)

    def _set_parse_content(self, v):
        self.parse_content = bool(v)

    def _set_fleet_send_batch_size(self, n=1024):
        self._fleet_send_batch_size = int(n)

    def _set_merge_by_lineid(self, merge_size=2):
        self.merge_by_lineid = True

    def load_into_memory(self, is_shuffle=False):
        self._data = self._read_files(self.filelist)
        self._loaded = True
        if is_shuffle:
            self.local_shuffle()

    def preload_into_memory(self, thread_num=None):
        if thread_num:
            self._set_thread(thread_num)
        self._pre = threading.Thread(target=self.load_into_memory)
        self._pre.start()

    def wait_preload_done(self):
        self._pre.join()

    def local_shuffle(self):
        random.shuffle(self._data)

    def global_shuffle(self, fleet=None, thread_num=12):
        """Redistribute instances uniformly at random over the trainers (an all-to-all over the
        default process group), then shuffle locally."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            self.local_shuffle()
            return
        W = dist.get_world_size()
        buckets = [[] for _ in range(W)]
        for inst in self._data:
            buckets[random.randrange(W)].append(inst)
        gathered = [None] * W
        dist.all_gather_object(gathered, buckets)  # every trainer's per-destination buckets
        me = dist.get_rank()
        self._data = [inst for r in range(W) for inst in gathered[r][me]]
        self.local_shuffle()

    def release_memory(self):
        self._data = []
        self._loaded = False

    def get_memory_data_size(self, fleet=None):
        n = len(self._data)
        return _sum_over_trainers(n) if fleet is not None else n

    def get_shuffle_data_size(self, fleet=None):
        return self.get_memory_data_size(fleet)

    def slots_shuffle(self, slots):
        """Shuffle the values of the named slots across instances (feature-importance evaluation)."""
        names = [m[0] for m in self._metas]
        for s in slots:
            vi = names.index(s)
            col = [inst[vi] for inst in self._data]
            random.shuffle(col)
            for inst, c in zip(self._data, col):
                inst[vi] = c

    def _iter_batches(self):
        if not self._loaded:
            raise RuntimeError("InMemoryDataset: call load_into_memory() before training")
        return self._batches(self._data)


def _sum_over_trainers(n):
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([n], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())
    return n


class QueueDataset(DatasetBase):
    """Streams the files (no in-memory stage, no shuffle)."""

    def init(self, **kwargs):
        super().init(**kwargs)

    def local_shuffle(self):
        raise NotImplementedError("QueueDataset streams its files and does not support local_shuffle; "
                                  "use InMemoryDataset")

    def global_shuffle(self, fleet=None):
        raise NotImplementedError("QueueDataset streams its files and does not support global_shuffle; "
                                  "use InMemoryDataset")

    def _iter_batches(self):
        pending = []
        for f in self.filelist:
            pending.extend(self._read_file(f))
            while len(pending) >= self.batch_size:
                yield self._batch_feed(pending[:self.batch_size])
                pending = pending[self.batch_size:]
        if pending:
            yield self._batch_feed(pending)


class FileInstantDataset(QueueDataset):
    pass


class DatasetFactory:
    """``DatasetFactory().create_dataset("InMemoryDataset")`` (legacy entry point)."""

    def create_dataset(self, datafeed_class="QueueDataset"):
        cls = {'InMemoryDataset': InMemoryDataset, 'QueueDataset': QueueDataset,
               'FileInstantDataset': FileInstantDataset}.get(datafeed_class)
        if cls is None:
            raise ValueError(f"datafeed class {datafeed_class} does not exist")
        return cls()
