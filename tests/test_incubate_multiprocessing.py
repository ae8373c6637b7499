"""paddle.incubate.multiprocessing: Tensors cross a Queue through shared memory (a write in the
child is seen by the parent), Parameters keep their attributes."""
import numpy as np

import paddle
import paddle.incubate.multiprocessing as mp


def _child(q, out):
    t = q.get()
    t._t.add_(1.0)  # in place on the shared pages
    p = q.get()
    out.put((p.name, bool(p.trainable), p.numpy().sum().item()))


def test_tensor_shared_across_processes():
    ctx = mp.get_context('spawn')
    q, out = ctx.Queue(), ctx.Queue()
    x = paddle.zeros([4, 4])
    w = paddle.create_parameter([3], 'float32', name='w0')
    w._t.data.fill_(2.0)
    proc = ctx.Process(target=_child, args=(q, out))
    proc.start()
    q.put(x)
    q.put(w)
    name, trainable, s = out.get(timeout=120)
    proc.join(60)
    assert proc.exitcode == 0
    np.testing.assert_array_equal(x.numpy(), np.ones((4, 4), 'float32'))
    assert name == 'w0' and trainable and s == 6.0
