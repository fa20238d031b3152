"""C5 matcher timing by path (diagnostic): shipped, unpruned column side, every column decided,
keyed epilogue."""
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'modify-sift-gpu_amd/python')
import numpy as np, sgpu
from sift_synth import synth_descriptors, quantize
ctx = sgpu.SiftContext(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
d1 = synth_descriptors(n, 5000)
d2 = synth_descriptors(n, 5001, base=d1, n_dup=min(20000, n // 2))
q1, q2 = quantize(d1), quantize(d2)
ref = None
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
REG = getattr(ctx, "DEBUG_MATCH_REGSTAGE", 0)
for name, flags, mbm in (("plain", 0, 1), ("plain_noprune", -1, 1),
                         ("full_columns", ctx.DEBUG_FULL_COLUMNS, 1),
                         ("keyed", ctx.DEBUG_KEYED_MATCH, 1), ("rows_only", 0, 0),
                         ("plain_reg", REG, 1), ("rows_reg", REG, 0)):
    if only and name not in only:
        continue
    ctx.set_match_prune(flags != -1)   # plain_noprune: every row of set 1 on the column side
    ctx.set_debug_flags(max(flags, 0))
    m = ctx.match(q1, q2, mbm=mbm)
    t = []
    for _ in range(10):
        m = ctx.match(q1, q2, mbm=mbm)
        t.append(ctx.timing()["match"])
    if mbm and ref is None:
        ref = m
    same = "" if not mbm else ("same pairs" if np.array_equal(m, ref) else "PAIRS DIFFER")
    print(f"{name}: min {min(t):.3f} ms median {np.median(t):.3f} ms, {len(m)} matches {same}", flush=True)
ctx.set_debug_flags(0)
