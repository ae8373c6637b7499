"""paddle.decomposition (reference: python/paddle/decomposition/decomp.py): composite-op
decomposition of static programs.  Our static programs are recorded at the torch-op level, so
they are already primitive; ``decompose`` returns the program's outputs unchanged."""


def decompose(program, src_vars, blacklist=frozenset(), whitelist=frozenset(), start_index=0, end_index=-1):
    return src_vars
