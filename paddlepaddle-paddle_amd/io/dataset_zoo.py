"""Legacy ``paddle.dataset`` readers (reference: python/paddle/dataset/*): backed by the
paddle.vision / paddle.text datasets, local files only."""


class mnist:  # noqa: N801
    @staticmethod
    def train(image_path=None, label_path=None):
        from ..vision.datasets import MNIST
        ds = MNIST(image_path, label_path, mode='train', backend='cv2')
        return lambda: ((img.reshape(-1) / 255.0, int(lab[0])) for img, lab in (ds[i] for i in range(len(ds))))

    test = train


class uci_housing:  # noqa: N801
    @staticmethod
    def train(data_file=None):
        from ..text import UCIHousing
        ds = UCIHousing(data_file, 'train')
        return lambda: (ds[i] for i in range(len(ds)))
