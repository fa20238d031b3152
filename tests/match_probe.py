"""Matcher timing probe (plain and guided) at C5 size, for rocprofv3 kernel traces:
    rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -- python3 tests/match_probe.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
import sgpu  # noqa: E402
from sift_synth import synth_descriptors, synth_guided_scene, quantize  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
variants = [int(v) for v in sys.argv[2:]] or [0]   # sgpu_debug_set_variant values to compare
ctx = sgpu.SiftContext()
d1 = synth_descriptors(n, 5000)
d2 = synth_descriptors(n, 5001, base=d1, n_dup=min(20000, n // 2))
q1, q2 = quantize(d1), quantize(d2)
g1, g2, l1, l2, H, F = synth_guided_scene(n, n, 5002)
for v in variants:
    sgpu.lib().sgpu_debug_set_variant(v)
    for name, fn in (("plain", lambda: ctx.match(q1, q2)),
                     ("guided", lambda: ctx.match_guided(g1, g2, l1, l2, H, F))):
        fn()
        t = []
        for _ in range(5):
            m = fn()
            t.append(ctx.timing()["match"])
        print(f"variant {v} {name}: {min(t):.3f} ms (min of 5), {len(m)} matches", flush=True)
sgpu.lib().sgpu_debug_set_variant(0)
