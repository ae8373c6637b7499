"""paddle.reader decorators (reference: python/paddle/reader/decorator.py)."""
import itertools
import queue
import random
import threading


def cache(reader):
    all_data = tuple(reader())

    def r():
        yield from all_data
    return r


def map_readers(func, *readers):
    def r():
        for items in zip(*[rd() for rd in readers]):
            yield func(*items)
    return r


def shuffle(reader, buf_size):
    def r():
        buf = []
        for e in reader():
            buf.append(e)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        random.shuffle(buf)
        yield from buf
    return r


def chain(*readers):
    def r():
        for rd in readers:
            yield from rd()
    return r


def compose(*readers, check_alignment=True):
    def r():
        its = [rd() for rd in readers]
        for items in (zip(*its) if check_alignment else itertools.zip_longest(*its)):
            out = []
            for it in items:
                out.extend(it if isinstance(it, tuple) else (it,))
            yield tuple(out)
    return r


def buffered(reader, size):
    """Prefetches up to ``size`` items on a background thread."""
    end = object()

    def r():
        q = queue.Queue(maxsize=size)

        def fill():
            for e in reader():
                q.put(e)
            q.put(end)
        threading.Thread(target=fill, daemon=True).start()
        while True:
            e = q.get()
            if e is end:
                return
            yield e
    return r


def firstn(reader, n):
    def r():
        yield from itertools.islice(reader(), n)
    return r


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    from concurrent.futures import ThreadPoolExecutor

    def r():
        with ThreadPoolExecutor(process_num) as ex:
            yield from ex.map(mapper, reader())
    return r


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    return chain(*readers)
