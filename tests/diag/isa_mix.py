"""Instruction mix of a kernel's innermost loop (CPU-side ISA check, no GPU):
  python tests/diag/isa_mix.py <file.s> <kernel-name substring>
The loop is the block from the last 'Loop Header' label to the branch back to it."""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read().splitlines()
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
body = text[start:end + 1]
hdr = [i for i, l in enumerate(body) if "Loop Header" in l]
h = hdr[-1]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if l.startswith(".LBB")}
# the latch: the last branch after the header whose target label lies at or before the header
back = max(i for i, l in enumerate(body) if i > h and "branch" in l and l.split()[-1] in labels
           and labels[l.split()[-1]] <= h)
h = labels[body[back].split()[-1]]
loop = [l.strip() for l in body[h:back + 1] if l.strip() and not l.strip().startswith((";", "."))]
c = Counter()
for l in loop:
    op = l.split()[0]
    c["all"] += 1
    c["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
      "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "scratch_", "flat_")) else "other"] += 1
    for k in ("v_pk_fma_f32", "v_mov", "v_cndmask", "s_waitcnt", "s_nop", "s_cbranch", "v_readlane", "global_load_lds"):
        if op.startswith(k):
            c[k] += 1
print(f"{sys.argv[2]}: loop {len(loop)} instructions:", dict(c))
