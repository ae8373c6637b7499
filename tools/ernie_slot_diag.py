"""Diagnostic: gradient storage of the ERNIE static step's parameters on the GPU (flat slots,
registry identity, gradients left after a step) and why the weight-gradient slot path is taken
or not."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], '--ernie-batch', '8']
    args = bench.parse()
    torch.cuda.set_device(0)
    from paddle.ops import matmul as HM
    from paddle.core.tensor import _PARAMS
    from paddle.parallel.flat_buffer import flat_grad_slot
    calls = {'ok': 0, 'fail': 0, 'why': {}}
    orig = HM.slot_wgrad

    def spy(x2, g2, w):
        r = orig(x2, g2, w)
        calls['ok' if r else 'fail'] += 1
        if not r:
            p = _PARAMS.get(id(w))
            why = 'no param' if p is None else ('other tensor' if p._t is not w else
                                               ('not flat' if '_flat' not in p.__dict__ else
                                                ('grad None' if p._t.grad is None else
                                                 ('slot None' if flat_grad_slot(p) is None else 'kernel'))))
            calls['why'][why] = calls['why'].get(why, 0) + 1
        return r
    HM.slot_wgrad = spy
    step, *_ = bench.build_ernie_static(args, 1, 0, torch.device('cuda', 0), False)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    print('slot_wgrad:', calls)
    ps = [p for p in _PARAMS.values()]
    print('registered params', len(ps), 'flat', sum('_flat' in p.__dict__ for p in ps),
          'grad None', sum(p._t.grad is None for p in ps), 'dtypes', {str(p._t.dtype) for p in ps})


if __name__ == '__main__':
    main()
