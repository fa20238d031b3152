"""Writes tests/golden/match_shard_states.npz on the GPU box: the sharded SiftMatch's per-rank
outputs of sgpu_match_shard_begin (row decisions + column state) for a 2-way split of set 1, and
the single-device sgpu_match pairs of the same sets, so that CPU tests can run the library's merge
(sgpu_match_shard_end) over gloo on real device shard states.
  python tests/make_shard_fixtures.py [out.npz]   (GPU; gpurun returns files under gpurun_out/)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "modify-sift-gpu_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import sgpu  # noqa: E402
from sift_dist import shard  # noqa: E402
from sift_synth import quantize, synth_descriptors  # noqa: E402


def main():
    n1, n2 = 3000, 2700
    d1 = synth_descriptors(n1, 6100)
    q1 = quantize(d1)
    q2 = quantize(synth_descriptors(n2, 6101, base=d1, n_dup=1100))
    ctx = sgpu.SiftContext(0)
    full = ctx.match(q1, q2)
    out = {"q1": q1, "q2": q2, "full": full}
    for r in range(2):
        s, e = shard(n1, r, 2)
        rows, cols = ctx.match_shard_begin(q1[s:e], s, q2)
        out[f"rows{r}"], out[f"cols{r}"] = rows, cols
        out[f"begin{r}"] = np.int32(s)
    ctx.close()
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden",
                                                               "match_shard_states.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(full)} pairs, shards {[len(out['rows0']), len(out['rows1'])]}")


if __name__ == "__main__":
    main()
