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


def _verify_worker(rank, world, port, per_rank, tamper, queue):
    import torch.distributed as dist
    import oracle_py
    from sift_dist import gather_records, image_digest, verify_records, verify_sample
    from sift_synth import synth_batch_fast
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # this rank's shard, as bench.py: images [rank B, (rank + 1) B) of seeds 3000 + global index
    imgs = synth_batch_fast(per_rank, 96, 80, 3000 + rank * per_rank)
    recs = np.array([image_digest(*oracle_py.extract(im)) for im in imgs], np.int32)
    if tamper and rank == 1:
        recs[-1, 1] ^= 1   # one descriptor bit of the last image, as a wrong rank would report
    allrec = gather_records(recs, dist)
    if rank == 0:
        sample = verify_sample(world, per_rank, 2)
        redo = {g: image_digest(*oracle_py.extract(synth_batch_fast(1, 96, 80, 3000 + g)[0]))
                for g in sample}
        queue.put(verify_records(allrec, redo))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("tamper", [False, True])
def test_gloo_world2_verify_exchange(tamper):
    """bench.py --verify's exchange over gloo (world size 2): every rank all-gathers (count,
    64-bit digest) per image, rank 0 recomputes the other rank's first and last images and
    compares -- verified on honest records, and the one flipped bit of a tampered record is
    caught (the oracle stands in for each rank's GPU here)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, 2, port, 3, tamper, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["images_gathered"] == 6 and res["recomputed"] == [3, 5]
    assert res["features_gathered"] > 0
    if tamper:
        assert not res["verified"] and res["mismatches"] == [5]
    else:
        assert res["verified"] and res["mismatches"] == []


def test_verify_sample_and_records():
    from sift_dist import verify_records, verify_sample
    assert verify_sample(1, 128, 2) == [0, 127]
    assert verify_sample(4, 128, 2) == [128, 255, 256, 383, 384, 511]
    recs = np.zeros((4, 3), np.int32)
    recs[2] = (7, -5, 9)
    assert verify_records(recs, {2: (7, -5, 9)})["verified"]
    assert not verify_records(recs, {2: (7, -5, 8)})["verified"]
    assert not verify_records(recs, {})["verified"]


def _fixture_merge_worker(rank, world, port, queue):
    import torch.distributed as dist
    from sift_dist import match_sharded_host
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    f = np.load(os.path.join(os.path.dirname(__file__), "golden", "match_shard_states.npz"))
    pairs = match_sharded_host(f[f"rows{rank}"], f[f"cols{rank}"], int(f[f"begin{rank}"]), dist)
    queue.put((rank, pairs.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_merge_of_device_shard_states():
    """The library's merge (sgpu_match_shard_end) over gloo, world size 2, on shard states that
    sgpu_match_shard_begin produced on an MI355X (tests/golden/match_shard_states.npz, written by
    tests/make_shard_fixtures.py): the ranks' pairs in rank order equal the device's own
    single-call sgpu_match pairs and the oracle's."""
    import torch.multiprocessing as mp
    import oracle_py
    path = os.path.join(os.path.dirname(__file__), "golden", "match_shard_states.npz")
    if not os.path.exists(path):
        pytest.skip("fixture not generated (tests/make_shard_fixtures.py on the GPU box)")
    f = np.load(path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fixture_merge_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.array(res[0] + res[1], np.int32).reshape(-1, 2)
    assert len(f["full"]) > 500
    np.testing.assert_array_equal(got, f["full"])
    np.testing.assert_array_equal(got, oracle_py.match(f["q1"], f["q2"]))
