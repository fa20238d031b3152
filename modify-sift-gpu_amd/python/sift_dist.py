"""Multi-GPU batch extraction: one process per GPU, images sharded, one collective.

Reference analogue: TestWin/MultiThreadSIFT.cpp:141-155 (one SiftGPU instance per device thread)
and the per-port server processes of ServerSiftGPU (ServerSiftGPU.cpp:156-194).  Here each rank
owns a contiguous shard of the batch and runs the whole hot path locally; the only exchange is one
all-gather of the per-image feature counts, from which every rank knows the global output layout
(image i's features start at offsets[i]).  On MI355X the all-gather is RCCL over xGMI inside
libsiftgpu (sgpu_comm_allgather_i32, used by bench.py); gather_counts below is the same exchange
through torch.distributed, used with gloo on CPU by the tests.
"""
from __future__ import annotations

import numpy as np


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, end) of n_total images for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_counts(local_counts: np.ndarray, n_total: int, dist, device=None) -> np.ndarray:
    """All-gather per-image feature counts of every rank's shard into the global [n_total]
    array (one collective; shards are padded to the largest shard size)."""
    import torch
    world = dist.get_world_size()
    width = max(shard(n_total, r, world)[1] - shard(n_total, r, world)[0] for r in range(world))
    buf = torch.zeros(width, dtype=torch.int32, device=device)
    buf[: len(local_counts)] = torch.from_numpy(np.ascontiguousarray(local_counts, np.int32))
    out = torch.zeros(width * world, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(out, buf)
    out = out.cpu().numpy().reshape(world, width)
    parts = []
    for r in range(world):
        s, e = shard(n_total, r, world)
        parts.append(out[r, : e - s])
    return np.concatenate(parts)


def global_offsets(counts: np.ndarray) -> np.ndarray:
    """offsets[i] = first global feature index of image i; offsets[n] = total."""
    off = np.zeros(len(counts) + 1, np.int64)
    np.cumsum(counts, out=off[1:])
    return off


def match_sharded_host(row_match: np.ndarray, col_best: np.ndarray, row_begin: int, dist,
                       distmax=0.7, ratiomax=0.8, mbm=1) -> np.ndarray:
    """Sharded SiftMatch exchange over torch.distributed (gloo on the host): all-gather every
    rank's column state ([n2][3] int32 from SiftContext.match_shard_begin) and finish this
    rank's rows (sgpu_match_shard_end).  The RCCL form of the same exchange is
    SiftContext.match_sharded."""
    import torch
    import sgpu
    world = dist.get_world_size()
    mine = torch.from_numpy(np.ascontiguousarray(col_best, np.int32).reshape(-1))
    out = torch.zeros(mine.numel() * world, dtype=torch.int32)
    dist.all_gather_into_tensor(out, mine)
    allc = out.numpy().reshape(world, -1, 3)
    return sgpu.match_shard_end(allc, row_match, row_begin, distmax, ratiomax, mbm)


# ---- self-verifying multi-GPU runs (bench.py --verify; SURVEY.md §4 (vi): the N-GPU output must
# equal the 1-GPU output image by image)

def image_digest(keys: np.ndarray, desc: np.ndarray | None) -> tuple[int, int, int]:
    """(feature count, low and high 32 bits of a 64-bit BLAKE2b digest of the image's key and
    descriptor bits) -- three int32 words that travel in one all-gather."""
    import hashlib
    h = hashlib.blake2b(digest_size=8)
    h.update(np.ascontiguousarray(keys, np.float32).tobytes())
    if desc is not None:
        h.update(np.ascontiguousarray(desc, np.float32).tobytes())
    v = int.from_bytes(h.digest(), "little")
    lo, hi = v & 0xffffffff, v >> 32
    as_i32 = lambda u: u - (1 << 32) if u >= (1 << 31) else u  # noqa: E731
    return int(len(keys)), as_i32(lo), as_i32(hi)


def verify_sample(world: int, per_rank: int, per_rank_images: int) -> list[int]:
    """Global image indices rank 0 recomputes: the first and last images of every other rank's
    shard (of its own shard when it runs alone), at most per_rank_images of each."""
    out = []
    ranks = range(1, world) if world > 1 else range(1)
    for r in ranks:
        first, last = r * per_rank, (r + 1) * per_rank - 1
        for g in sorted({first, last})[:per_rank_images]:
            out.append(g)
    return out


def verify_records(records: np.ndarray, recomputed: dict[int, tuple[int, int, int]]) -> dict:
    """Compare the all-gathered per-image records ([n_images][3] int32: count, digest lo, hi)
    with rank 0's recomputation of a sample {global index: record}."""
    records = np.asarray(records, np.int32).reshape(-1, 3)
    bad = [g for g, rec in sorted(recomputed.items()) if tuple(int(x) for x in records[g]) != tuple(rec)]
    return {"verified": not bad and len(recomputed) > 0, "images_gathered": int(len(records)),
            "recomputed": sorted(recomputed), "mismatches": bad,
            "features_gathered": int(records[:, 0].sum())}


def gather_records(local: np.ndarray, dist) -> np.ndarray:
    """All-gather every rank's [B][3] int32 records over torch.distributed (gloo on the host; the
    RCCL form is SiftContext.allgather_i32) -> [world * B][3] in rank order."""
    import torch
    world = dist.get_world_size()
    mine = torch.from_numpy(np.ascontiguousarray(local, np.int32).reshape(-1))
    out = torch.zeros(mine.numel() * world, dtype=torch.int32)
    dist.all_gather_into_tensor(out, mine)
    return out.numpy().reshape(-1, 3)
