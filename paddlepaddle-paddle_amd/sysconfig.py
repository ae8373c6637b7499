"""paddle.sysconfig (reference: python/paddle/sysconfig.py)."""
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def get_include():
    return os.path.join(_HERE, 'csrc')


def get_lib():
    return os.path.join(_HERE, '_lib')
