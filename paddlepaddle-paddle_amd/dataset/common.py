"""paddle.dataset.common (reference: python/paddle/dataset/common.py): DATA_HOME, md5, the
(offline) download resolver, split / cluster_files_reader."""
import glob
import hashlib
import os
import pickle

DATA_HOME = os.environ.get('PADDLE_DATA_HOME', os.path.join(os.path.expanduser('~'), '.cache', 'paddle', 'dataset'))

__all__ = []


def must_mkdirs(path):
    os.makedirs(path, exist_ok=True)


def md5file(fname):
    h = hashlib.md5()
    with open(fname, 'rb') as f:
        for chunk in iter(lambda: f.read(4096), b''):
            h.update(chunk)
    return h.hexdigest()


def download(url, module_name, md5sum=None, save_name=None):
    """Resolve DATA_HOME/module_name/<file name of url> — present locally or an error (no network).
    A given md5sum is checked."""
    path = os.path.join(DATA_HOME, module_name, save_name or url.split('/')[-1])
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: there is no network access here, place the file there by hand")
    if md5sum and md5file(path) != md5sum:
        raise RuntimeError(f"{path}: md5 mismatch")
    return path


def local(module_name, file_name):
    return download(file_name, module_name)


def fetch_all():
    raise RuntimeError("fetch_all needs network access")


def split(reader, line_count, suffix="%05d.pickle", dumper=pickle.dump):
    """Write the reader's samples in files of ``line_count`` samples each (these files are written
    and read back by this process only)."""
    if not callable(dumper):
        raise TypeError("dumper should be callable.")
    lines, idx = [], 0
    for i, d in enumerate(reader()):
        lines.append(d)
        if i >= line_count and i % line_count == 0:
            with open(suffix % idx, 'wb') as f:
                dumper(lines, f)
            lines, idx = [], idx + 1
    if lines:
        with open(suffix % idx, 'wb') as f:
            dumper(lines, f)


def cluster_files_reader(files_pattern, trainer_count, trainer_id, loader=pickle.load):
    """Reader over the files of ``files_pattern`` assigned to this trainer (file i goes to trainer
    i % trainer_count); ``loader`` reads one file's sample list (files this job wrote itself)."""
    def reader():
        if not callable(loader):
            raise TypeError("loader should be callable.")
        for i, fn in enumerate(sorted(glob.glob(files_pattern))):
            if i % trainer_count == trainer_id:
                with open(fn, 'rb') as f:
                    yield from loader(f)
    return reader
