"""paddle.utils.download (reference: python/paddle/utils/download.py).  No network here: only
local paths / already-cached files resolve; anything else raises a clear error."""
import os

WEIGHTS_HOME = os.path.expanduser(os.environ.get('PADDLE_WEIGHTS_HOME', '~/.cache/paddle/hapi/weights'))


def is_url(path):
    return str(path).startswith(('http://', 'https://'))


def get_path_from_url(url, root_dir=None, md5sum=None, check_exist=True, decompress=True, method='get'):
    root_dir = root_dir or WEIGHTS_HOME
    if not is_url(url):
        return url
    cached = os.path.join(root_dir, url.split('/')[-1])
    if os.path.exists(cached):
        return cached
    raise RuntimeError(f"cannot download {url}: no network access (place the file at {cached})")


def get_weights_path_from_url(url, md5sum=None):
    return get_path_from_url(url, WEIGHTS_HOME, md5sum)
