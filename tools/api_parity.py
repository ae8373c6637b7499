"""Public-API parity against the reference: for every reference module that declares ``__all__``
(read with ``ast`` from /root/reference/python/paddle, nothing imported from it), import the same
module path from this package and list the names it lacks.

usage: python tools/api_parity.py [--all]   (--all: also print modules with no gap)
"""
import ast
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = '/root/reference/python/paddle'
SKIP_PARTS = {'tests', 'test', 'libs', 'proto', 'cinn', 'pir', '_typing', 'base', 'fluid'}


def ref_all(path):
    try:
        tree = ast.parse(open(path, encoding='utf-8').read())
    except (SyntaxError, UnicodeDecodeError):
        return None
    for node in tree.body:
        targets = []
        if isinstance(node, ast.Assign):
            targets = node.targets
        elif isinstance(node, ast.AnnAssign):
            targets = [node.target]
        for t in targets:
            if isinstance(t, ast.Name) and t.id == '__all__':
                try:
                    v = ast.literal_eval(node.value)
                except ValueError:
                    return None
                return [n for n in v if isinstance(n, str)]
    return None


def main(show_all=False):
    import paddle  # noqa: F401
    total = missing_total = 0
    rows = []
    for dirpath, dirnames, filenames in os.walk(REF):
        rel = os.path.relpath(dirpath, REF)
        parts = [] if rel == '.' else rel.split(os.sep)
        if any(p in SKIP_PARTS or p.startswith('_') for p in parts):
            continue
        if '__init__.py' not in filenames:
            continue
        names = ref_all(os.path.join(dirpath, '__init__.py'))
        if not names:
            continue
        mod = '.'.join(['paddle'] + parts)
        try:
            m = importlib.import_module(mod)
        except Exception as e:  # noqa: BLE001
            rows.append((mod, len(names), names, f'IMPORT FAILED: {type(e).__name__}: {e}'))
            total += len(names)
            missing_total += len(names)
            continue
        miss = [n for n in names if not hasattr(m, n)]
        total += len(names)
        missing_total += len(miss)
        rows.append((mod, len(names), miss, None))
    for mod, n, miss, err in sorted(rows):
        if err:
            print(f'{mod:55s} {n:4d}  {err}')
        elif miss or show_all:
            print(f'{mod:55s} {n:4d}  missing {len(miss)}: {" ".join(miss[:40])}')
    print(f'TOTAL reference __all__ names {total}, missing {missing_total} '
          f'({100.0 * (total - missing_total) / max(total, 1):.1f} % present)')


if __name__ == '__main__':
    main('--all' in sys.argv)
