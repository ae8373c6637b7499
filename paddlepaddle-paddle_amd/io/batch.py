"""paddle.batch (reference: python/paddle/batch.py): batches a sample reader."""


def batch(reader, batch_size, drop_last=False):
    if batch_size <= 0:
        raise ValueError("batch_size should be a positive integer")

    def batch_reader():
        b = []
        for item in reader():
            b.append(item)
            if len(b) == batch_size:
                yield b
                b = []
        if b and not drop_last:
            yield b
    return batch_reader
