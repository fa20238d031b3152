"""Row-side pairs of the LDS-DMA matcher vs the register-staged one for row counts that give
1..6 tiles per column chunk (diagnostic)."""
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu
from sift_synth import synth_descriptors, quantize
ctx = sgpu.SiftContext(0)
d1 = synth_descriptors(20000, 5000)
d2 = synth_descriptors(20000, 5001, base=d1, n_dup=8000)
q1, q2 = quantize(d1), quantize(d2)
R = ctx.DEBUG_MATCH_REGSTAGE
for n in (20000, 12000, 8000, 4000, 2000, 1000, 300):
    out = []
    for rep in range(3):
        ctx.set_debug_flags(0)
        a = ctx.match(q1[:n], q2, 0.9, 0.8, 0)
        ctx.set_debug_flags(R)
        b = ctx.match(q1[:n], q2, 0.9, 0.8, 0)
        out.append((len(a), len(b), np.array_equal(a, b)))
    print(n, out)
