"""A/B wrapper: run bench.py in-process with the bias+activation launch knobs set first.
usage: python tools/ab_act.py FWD_BLOCKS FWD_UNROLL CS_BLOCKS [bench args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == '__main__':
    fb, fu, cs = (int(v) for v in sys.argv[1:4])
    import paddle  # noqa: F401
    from paddle.ops import _native
    _native._load()
    _native.lib.pa_act_fwd_tune(fb, fu)
    _native.lib.pa_act_cs_tune(cs)
    print(f"act knobs: fwd blocks={fb} unroll={fu} colsum blocks={cs}", flush=True)
    sys.argv = [os.path.join(ROOT, 'bench.py')] + sys.argv[4:]
    runpy.run_path(sys.argv[0], run_name='__main__')
