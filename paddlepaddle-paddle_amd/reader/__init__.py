"""paddle.reader: legacy sample-reader decorators (reference: python/paddle/reader/decorator.py);
implemented in io/reader.py."""
from ..io.reader import (cache, map_readers, shuffle, chain, compose, buffered, firstn, xmap_readers,  # noqa: F401
                         multiprocess_reader)
from ..io import reader as decorator  # noqa: F401

__all__ = []
