"""paddle.dataset: the legacy reader-creator corpora (reference: python/paddle/dataset/*).

Each module returns reader creators (zero-argument callables yielding samples) over the
paddle.vision / paddle.text dataset classes.  Nothing is downloaded: the archives are looked up
where the reference's downloader would have put them, ``common.DATA_HOME/<module>/<file>``
(``$PADDLE_DATA_HOME``, default ``~/.cache/paddle/dataset``), and a missing file raises.
"""
from . import common, image, mnist, cifar, uci_housing, imdb, imikolov, movielens, conll05, wmt14, wmt16  # noqa: F401
from . import flowers, voc2012  # noqa: F401

__all__ = []
