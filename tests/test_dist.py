"""Multi-rank batch path on CPU (gloo, world size 2): sharding, the count all-gather and the
global offsets match a single-process run image by image."""
import os
import socket

import numpy as np
import pytest

from sift_dist import shard, global_offsets


def test_shard_covers_batch():
    for n in [1, 5, 8, 1024, 1023]:
        for world in [1, 2, 3, 8]:
            ranges = [shard(n, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, queue):
    import torch.distributed as dist
    import oracle_py
    from sift_dist import gather_counts, shard
    from sift_synth import synth_image
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard(n_total, rank, world)
    counts = np.array([len(oracle_py.extract(synth_image(96, 80, 100 + i))[0]) for i in range(s, e)],
                      np.int32)
    allc = gather_counts(counts, n_total, dist)
    queue.put((rank, allc.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [4, 5])
def test_gloo_world2_counts(n_total):
    import torch.multiprocessing as mp
    import oracle_py
    from sift_synth import synth_image
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    serial = [len(oracle_py.extract(synth_image(96, 80, 100 + i))[0]) for i in range(n_total)]
    assert res[0] == serial and res[1] == serial
    off = global_offsets(np.array(serial))
    assert off[-1] == sum(serial) and off[0] == 0


def _match_worker(rank, world, port, queue):
    import torch.distributed as dist
    from test_oracle import np_shard_state
    from sift_dist import match_sharded_host, shard
    from sift_synth import synth_descriptors, quantize
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q1 = quantize(synth_descriptors(300, 5200))
    q2 = quantize(synth_descriptors(280, 5201, base=synth_descriptors(300, 5200), n_dup=120))
    s, e = shard(len(q1), rank, world)
    rows, state = np_shard_state(q1[s:e], s, q2)     # what begin returns on a GPU rank
    pairs = match_sharded_host(rows, state, s, dist)
    queue.put((rank, pairs.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_match():
    """Sharded SiftMatch over gloo (world size 2): each rank's pairs, concatenated in rank
    order, are the single-process matcher's."""
    import torch.multiprocessing as mp
    import oracle_py
    from sift_synth import synth_descriptors, quantize
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_match_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    q1 = quantize(synth_descriptors(300, 5200))
    q2 = quantize(synth_descriptors(280, 5201, base=synth_descriptors(300, 5200), n_dup=120))
    full = oracle_py.match(q1, q2)
    got = np.array(res[0] + res[1], np.int32).reshape(-1, 2)
    assert len(full) > 30
    np.testing.assert_array_equal(got, full)
