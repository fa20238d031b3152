"""Pair counts of the keyless matcher's LDS-DMA kernel against the register-staged one on the
parity test's cases, per debug flag set (diagnostic)."""
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu
from sift_synth import synth_descriptors, quantize
import oracle_py as O
ctx = sgpu.SiftContext(0)
d1 = synth_descriptors(20000, 5000)
d2 = synth_descriptors(20000, 5001, base=d1, n_dup=8000)
q1, q2 = quantize(d1), quantize(d2)
small = (quantize(synth_descriptors(700, 8)), quantize(synth_descriptors(129, 9)))
R = ctx.DEBUG_MATCH_REGSTAGE
F = ctx.DEBUG_FULL_COLUMNS
for name, (a, b) in (("20k", (q1, q2)), ("700x129", small), ("129x700", small[::-1])):
    for mbm in (0, 1):
        res = {}
        for fl in (0, R, F, F | R):
            ctx.set_debug_flags(fl)
            res[fl] = ctx.match(a, b, 0.9, 0.8, mbm)
        ctx.set_debug_flags(0)
        ref = O.match(a, b, 0.9, 0.8, mbm) if len(a) < 5000 else None
        print(name, "mbm", mbm, {k: len(v) for k, v in res.items()},
              "ref", None if ref is None else len(ref),
              "dma==reg", np.array_equal(res[0], res[R]), "full dma==reg", np.array_equal(res[F], res[F | R]))
