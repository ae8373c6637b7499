"""Model-parallel RNG state tracker (reference: python/paddle/distributed/fleet/layers/mpu/random.py).

Dropout inside a tensor-parallel region must differ across mp ranks (local seed) while
dropout on replicated activations must agree (global seed); named RNG states are swapped in
and out around ``rng_state(name)`` blocks.
"""
import contextlib

import torch

MODEL_PARALLEL_RNG = 'model_parallel_rng'


class RNGStatesTracker:
    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def add(self, name, seed):
        if seed in self.seeds_:
            raise ValueError(f'seed {seed} already exists')
        if name in self.states_:
            raise ValueError(f'state {name} already exists')
        self.seeds_.add(seed)
        cpu = torch.get_rng_state()
        cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        torch.manual_seed(seed)
        self.states_[name] = (torch.get_rng_state(), torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
        torch.set_rng_state(cpu)
        if cuda is not None:
            torch.cuda.set_rng_state(cuda)

    def get_states_tracker(self):
        return dict(self.states_)

    def set_states_tracker(self, states):
        self.states_ = dict(states)

    @contextlib.contextmanager
    def rng_state(self, name=MODEL_PARALLEL_RNG):
        if name not in self.states_:
            raise ValueError(f'state {name} does not exist')
        cpu = torch.get_rng_state()
        cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        s_cpu, s_cuda = self.states_[name]
        torch.set_rng_state(s_cpu)
        if s_cuda is not None:
            torch.cuda.set_rng_state(s_cuda)
        try:
            yield
        finally:
            self.states_[name] = (torch.get_rng_state(),
                                  torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
            torch.set_rng_state(cpu)
            if cuda is not None:
                torch.cuda.set_rng_state(cuda)


_TRACKER = RNGStatesTracker()


def get_rng_state_tracker():
    return _TRACKER


def model_parallel_random_seed(seed=None):
    import random
    from ... import _inited, get_hybrid_communicate_group
    hcg = get_hybrid_communicate_group() if _inited() else None
    rank = hcg.get_model_parallel_rank() if hcg else 0
    global_seed = seed if seed is not None else random.randint(0, 10000)
    local_seed = global_seed + 1024 + rank * 100
    _TRACKER.reset()
    _TRACKER.add(MODEL_PARALLEL_RNG, local_seed)
    torch.manual_seed(global_seed)


def determinate_seed(rng_name):
    return 0


def dropout(x, p=0.5, axis=None, rng_name=None, training=True, mode="upscale_in_train", name=None):
    from .....nn import functional as F
    if rng_name is None or rng_name not in _TRACKER.states_:
        return F.dropout(x, p, axis, training, mode)
    with _TRACKER.rng_state(rng_name):
        return F.dropout(x, p, axis, training, mode)
