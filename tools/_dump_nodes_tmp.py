import os, sys; sys.path.insert(0, os.getcwd())
import sys; sys.path.insert(0, 'tests')
import paddle
from paddle.static import ir_passes as IP
from test_ir_passes import _build
main, loss, logits = _build(True, 0.1)
for i, n in enumerate(main.nodes):
    k = IP._kind(n)
    name = getattr(n.target, '__name__', type(n.target).__name__) if n.kind == 'torch' else n.kind
    args = [('R%d' % a.vid) if type(a).__name__ == 'Ref' else type(a).__name__ for a in n.args]
    if 40 <= i <= 110:
        print(i, n.kind, k, name, args, n.kwargs if len(str(n.kwargs)) < 80 else '...', n.outs)
