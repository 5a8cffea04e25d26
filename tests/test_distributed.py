"""Row-sharded search (brickrec.distributed.ShardedIndex) at world_size 2 over gloo on CPU:
every rank's merged result equals the unsharded oracle for semantic, similar (rank-0
drop across shards), CF (exclusions) and hybrid (union blend), with a constraint mask."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N, D, R_, B, K = 997, 24, 8, 5, 7


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rng = np.random.default_rng(5)
    x = rng.standard_normal((N, D)).astype(np.float32)
    x[::97] = x[3]                      # duplicate rows: equal scores, ties by id
    f = (0.1 * rng.standard_normal((N, R_))).astype(np.float32)
    q = rng.standard_normal((B, D)).astype(np.float32)
    u = (0.1 * rng.standard_normal((B, R_))).astype(np.float32)
    mask = rng.random(N) < 0.6
    excl = rng.random((B, N)) < 0.1
    items = np.array([3, 10, 500, 996, 499])
    return x, f, q, u, mask, excl, items


def _worker(rank, world, port, out_q):
    import torch
    import torch.distributed as dist
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "brickbrain-rec-engine_amd"))
    from _oracle_shard import OracleShard
    from brickrec.distributed import ShardedIndex
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x, f, q, u, mask, excl, items = _data()
        si = ShardedIndex(N, index_factory=OracleShard)
        si.upload_items(x)
        si.upload_cf(f)
        res = {}
        res["semantic"] = si.search("semantic", K, q_rows=torch.from_numpy(q), mask=mask)
        res["similar"] = si.search("similar", K, q_items=items, mask=mask)
        res["cf"] = si.search("cf", K, q_cf=torch.from_numpy(u), excl=excl, mask=mask)
        res["hybrid"] = si.search("hybrid", K, q_items=items, q_cf=torch.from_numpy(u), excl=excl, mask=mask)
        # the scale interface: per-rank bitsets built once (mask sliced once, rated ids
        # scattered on the rank's device), passed to every search as they are
        mb = si.mask_bits(mask)
        eb = si.excl_bits([np.flatnonzero(excl[b]) for b in range(excl.shape[0])])
        assert mb.dtype == torch.int32 and tuple(mb.shape) == (si.words,)
        assert eb.dtype == torch.int32 and tuple(eb.shape) == (excl.shape[0], si.words)
        res["semantic/bits"] = si.search("semantic", K, q_rows=torch.from_numpy(q), mask=mb)
        res["similar/bits"] = si.search("similar", K, q_items=items, mask=mb)
        res["cf/bits"] = si.search("cf", K, q_cf=torch.from_numpy(u), excl=eb, mask=mb)
        res["hybrid/bits"] = si.search("hybrid", K, q_items=items, q_cf=torch.from_numpy(u), excl=eb, mask=mb)
        # pipelined merge (query chunks, each chunk's key gather in flight behind the next
        # chunk's local search): the same lists for every chunking
        res["semantic/pipe2"] = si.search("semantic", K, q_rows=torch.from_numpy(q), mask=mb, pipeline=2)
        res["hybrid/pipe3"] = si.search("hybrid", K, q_items=items, q_cf=torch.from_numpy(u), excl=eb, mask=mb,
                                        pipeline=3)
        out_q.put((rank, {m: tuple(t.numpy() for t in v) for m, v in res.items()}))
    finally:
        dist.destroy_process_group()


def _reference():
    """Unsharded oracle lists per mode for _data(): semantic, similar (rank 0 dropped, mask),
    CF (rated skipped, mask) and the hybrid union blend of their top-2k lists."""
    from oracle import restatement as R
    x, f, q, u, mask, excl, items = _data()
    xn = R.normalize_rows(x.astype(np.float64)).astype(np.float32)
    ref = {}
    for b in range(B):
        sim = (xn @ R.normalize_rows(q[b:b + 1].astype(np.float64))[0].astype(np.float32)).astype(np.float32)
        ref.setdefault("semantic", []).append(R.topk_indices(sim, K, mask))
        s2 = (xn @ xn[items[b]]).astype(np.float32)
        drop = int(np.flatnonzero(s2 == s2.max())[0])
        ok = mask.copy()
        ok[drop] = False
        ci, cs = R.topk_indices(s2, 2 * K, ok)
        ref.setdefault("similar", []).append((ci[:K], cs[:K]))
        fs = (f @ u[b]).astype(np.float32)
        fi, fsc = R.topk_indices(fs, 2 * K, mask & ~excl[b])
        ref.setdefault("cf", []).append((fi[:K], fsc[:K]))
        ref.setdefault("hybrid", []).append(R.union_blend(ci, cs, fi, fsc, 0.4, 0.6, K))
    return ref


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_matches_unsharded(world):
    from oracle import restatement as R
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q_)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q_.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _reference()
    for rank in range(world):
        for mode, (sc, ids, cnt) in outs[rank].items():
            for b in range(B):
                ri, rs = ref[mode.split("/")[0]][b]
                assert list(ids[b][: cnt[b]]) == list(ri), (rank, mode, b, ids[b], ri)
                np.testing.assert_allclose(sc[b][: cnt[b]], rs, atol=1e-6)
    # identical on every rank
    for mode in outs[0]:
        for a, b_ in zip(outs[0][mode], outs[1][mode]):
            np.testing.assert_array_equal(a, b_)


def test_shard_bounds_cover_rows():
    from brickrec.distributed import shard_bounds
    for n in (1, 7, 1000, 25216):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _worker_small(rank, world, port, out_q):
    """5 items over 4 ranks: per-rank blocks of 2, 2, 1 and 0 rows (rank 3 is empty)."""
    import torch
    import torch.distributed as dist
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "brickbrain-rec-engine_amd"))
    from _oracle_shard import OracleShard
    from brickrec.distributed import ShardedIndex
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        x, f, q, u = _small_data()
        si = ShardedIndex(5, index_factory=OracleShard)
        assert si.empty == (rank == 3)
        si.upload_items(x)
        si.upload_cf(f)
        res = {"semantic": si.search("semantic", 3, q_rows=torch.from_numpy(q)),
               "similar": si.search("similar", 3, q_items=np.array([4, 0])),
               "hybrid": si.search("hybrid", 2, q_items=np.array([4, 0]), q_cf=torch.from_numpy(u))}
        out_q.put((rank, {m: tuple(t.numpy() for t in v) for m, v in res.items()}))
    finally:
        dist.destroy_process_group()


def _small_data():
    rng = np.random.default_rng(11)
    return (rng.standard_normal((5, 6)).astype(np.float32), (0.1 * rng.standard_normal((5, 3))).astype(np.float32),
            rng.standard_normal((2, 6)).astype(np.float32), (0.1 * rng.standard_normal((2, 3))).astype(np.float32))


def test_empty_shard_world4():
    """N < P·ceil(N/P): the last rank holds no rows, contributes empty lists, and still
    returns the unsharded results (empty shards used to fail in upload)."""
    from oracle import restatement as R
    from brickrec.distributed import shard_bounds
    assert shard_bounds(5, 4, 3) == (5, 5)
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_small, args=(r, 4, port, q_)) for r in range(4)]
    for p in procs:
        p.start()
    outs = dict(q_.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x, f, q, u = _small_data()
    xn = R.normalize_rows(x.astype(np.float64)).astype(np.float32)
    for b in range(2):
        sim = (xn @ R.normalize_rows(q[b:b + 1].astype(np.float64))[0].astype(np.float32)).astype(np.float32)
        ri, rs = R.topk_indices(sim, 3)
        sc, ids, cnt = outs[0]["semantic"]
        assert list(ids[b][: cnt[b]]) == list(ri)
        it = [4, 0][b]
        s2 = (xn @ xn[it]).astype(np.float32)
        ok = np.ones(5, bool)
        ok[R.rank0(s2)] = False
        ci, cs = R.topk_indices(s2, 4, ok)
        sc, ids, cnt = outs[0]["similar"]
        assert list(ids[b][: cnt[b]]) == list(ci[:3])
        fi, fs = R.topk_indices((f @ u[b]).astype(np.float32), 4)
        hi, hs = R.union_blend(ci, cs, fi, fs, 0.4, 0.6, 2)
        sc, ids, cnt = outs[0]["hybrid"]
        assert list(ids[b][: cnt[b]]) == list(hi)
    for r in range(1, 4):
        for mode in outs[0]:
            for a, b_ in zip(outs[0][mode], outs[r][mode]):
                np.testing.assert_array_equal(a, b_)


def _single_rank_index(n):
    """A ShardedIndex of one gloo rank over OracleShard (its own process group)."""
    import socket
    import torch.distributed as dist
    from _oracle_shard import OracleShard
    from brickrec.distributed import ShardedIndex
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    return ShardedIndex(n, index_factory=OracleShard)


def test_local_bits_rejects_foreign_packed_words():
    """packed words must be this rank's — a bitset of the wrong length (global,
    another rank's, or a uint32 word array of another size) raises instead of reaching the
    kernel; bool arrays are packed; int32 / uint32 words of the right shape pass through."""
    import torch
    si = _single_rank_index(100)
    W = si.words
    good = torch.zeros(W, dtype=torch.int32)
    assert si._local_bits(good, False).shape == (W,)
    assert si._local_bits(np.zeros(W, np.uint32), False).dtype == torch.int32
    assert si._local_bits(np.zeros((3, W), np.uint32), True).shape == (3, W)
    assert si._local_bits(np.ones(100, bool), False).shape == (W,)
    # plain Python lists: packed like the arrays they stand for
    assert np.array_equal(si._local_bits([True] * 100, False).numpy(), si._local_bits(np.ones(100, bool), False).numpy())
    assert si._local_bits([[False] * 100] * 2, True).shape == (2, W)
    with pytest.raises(ValueError):
        si._local_bits([True] * 77, False)
    for bad, rows in ((torch.zeros(W + 1, dtype=torch.int32), False), (np.zeros(W * 2, np.uint32), False),
                      (torch.zeros((2, W), dtype=torch.int32), False), (np.zeros(W, np.int32), True),
                      (torch.zeros(W, dtype=torch.int64), False), (np.ones(77, bool), False)):
        with pytest.raises(ValueError):
            si._local_bits(bad, rows)


def test_excl_bits_tensor_repeats_count_once():
    """a repeated id in a padded [B, m] tensor sets its bit once (the scatter adds,
    so a duplicate would carry into the next bit)."""
    import torch
    si = _single_rank_index(100)
    ids = torch.tensor([[5, 5, 7, -1], [31, 31, 31, 0]])
    w = si.excl_bits(ids).numpy().view(np.uint32)
    assert w[0, 0] == (1 << 5) | (1 << 7)
    assert w[1, 0] == (1 << 31) | 1
    ref = si.excl_bits([[5, 7], [0, 31]]).numpy()
    assert np.array_equal(w.view(np.int32), ref)
