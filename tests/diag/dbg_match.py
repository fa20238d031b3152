import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu, oracle_py as O
from sift_synth import synth_descriptors, quantize
ctx = sgpu.SiftContext(0)
n1, n2, dup = 5000, 129, 50
d1 = synth_descriptors(n1, 10 * n1 + n2)
d2 = synth_descriptors(n2, 10 * n2 + n1 + 1, base=d1, n_dup=dup)
q1, q2 = quantize(d1), quantize(d2)
for mbm in (0, 1):
    a = ctx.match(q1, q2, mbm=mbm)
    b = O.match(q1, q2, mbm=mbm)
    sa = set(map(tuple, a.tolist())); sb = set(map(tuple, b.tolist()))
    print("mbm", mbm, len(a), len(b), "only gpu", sorted(sa - sb)[:10], "only oracle", sorted(sb - sa)[:10])
    for (i, j) in sorted(sb - sa)[:3]:
        dots = q1[i].astype(np.int64) @ q2.astype(np.int64).T
        o = np.argsort(-dots)[:3]
        print(" row", i, "oracle j", j, "top cols", o, dots[o])
