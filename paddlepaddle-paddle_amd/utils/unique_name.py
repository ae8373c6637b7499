"""paddle.utils.unique_name (reference: python/paddle/utils/unique_name.py)."""
import collections
import contextlib


class UniqueNameGenerator:
    def __init__(self, prefix=''):
        self.ids = collections.defaultdict(int)
        self.prefix = prefix

    def __call__(self, key):
        i = self.ids[key]
        self.ids[key] += 1
        return f"{self.prefix}{key}_{i}"


_generator = UniqueNameGenerator()


def generate(key):
    return _generator(key)


def generate_with_ignorable_key(key):
    return _generator(key)


def switch(new_generator=None):
    global _generator
    old = _generator
    _generator = new_generator or UniqueNameGenerator()
    return old


@contextlib.contextmanager
def guard(new_generator=None):
    if isinstance(new_generator, str):
        new_generator = UniqueNameGenerator(new_generator)
    old = switch(new_generator)
    try:
        yield
    finally:
        switch(old)
