"""Row-sharded item index across the GPUs of a node, for ≥1M-item indexes.

Layout:

* Item rows are split into P contiguous blocks of ⌈N/P⌉. Rank r owns rows [lo, hi) and
  builds its ``ItemIndex`` with ``id_offset = lo``, so its candidate keys carry global ids.
* CF factors, attribute columns and mask bits shard with the same rows.
* Queries, user factors and weights are replicated.

One search is:

1. Each rank runs a local ``bb_search`` with ``BB_Q_OUT_KEYS``. That gives per-side
   candidate lists of u64 keys, ``(ord(score) << 32) | (0xFFFFFFFF − gid)``, plus its
   unmasked arg-max key. The lists are top-K for semantic/CF, K+1 for similar (rank-0
   drop) and 2K+1 per side for hybrid.
2. **The only exchange:** one all-gather of the keys (B·sides·K_int·8 bytes per rank) and
   the max keys. The backend is RCCL over xGMI for ``nccl``, and ``gloo`` in CPU tests.
3. Each rank runs ``bb_finalize`` over the P lists: merge, global rank-0 drop, truncate,
   hybrid union blend. Because keys order by (score desc, id asc), the result does not
   depend on P.

Similar-sets queries name a liked set by global id, but only the owning shard holds that
row. The ranks therefore first assemble the query rows: each rank fetches the rows it owns
(``bb_get_rows``) and an all-reduce(sum) fills in the rest. Then every shard scans with
the same ``q_rows``, which is ``feat_matrix[target]`` (recommendation_system.py:213).

A rank whose block is empty (N < P·⌈N/P⌉ leaves the last ranks without rows, e.g. N=5 on
4 ranks) uploads nothing and contributes empty key lists (key 0 = empty slot) to the
gather; it still runs the merge, so every rank returns the same results.

Masks and exclusions cross the interface as per-rank device bitsets: ``mask_bits`` (a
predicate evaluated on the rank's own attribute columns by ``bb_eval_mask``, or a global
bool array sliced once) and ``excl_bits`` (per-query item-id lists, e.g. rated sets,
scattered into [B, words] on the device).  ``search`` takes them as they are — no
global [N] / [B, N] host array is sliced, packed or copied per call.  Global host arrays
are still accepted for small cases (tests), at that per-call cost.

At 25K items the index does not shard (39 MB); ``bench.py --gpus N`` runs replicas.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def _all_gather(t, group, world, async_op=False):
    """Gather equal-shape tensors -> [world, *t.shape] (one buffer with nccl/RCCL).  With
    async_op the collective is only enqueued (RCCL: on its own stream, after the work already
    on the current stream) and (out, work) comes back; work.wait() orders the current stream
    after it."""
    import torch
    import torch.distributed as dist
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        w = dist.all_gather_into_tensor(out, t.contiguous(), group=group, async_op=async_op)
    else:
        w = dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group, async_op=async_op)
    return (out, w) if async_op else out


def _gather_lists(keys, maxk, group, world, async_op=False):
    """The merge's one exchange: the key lists [sides, B, k_int] and max keys [B] of every
    rank as ONE all-gather of a packed int64 buffer (round 6: was two collectives).  Returns a
    function giving ([P, sides, B, k_int], [P, B]) once the gather has landed."""
    import torch
    nk = keys.numel()
    flat = torch.cat([keys.reshape(-1), maxk.reshape(-1)])
    res = _all_gather(flat, group, world, async_op)
    out, work = res if async_op else (res, None)

    def finish():
        if work is not None:
            work.wait()
        return (out[:, :nk].reshape((world,) + tuple(keys.shape)).contiguous(),
                out[:, nk:].reshape(world, maxk.shape[0]).contiguous())
    return finish


class ShardedIndex:
    """The rank-local shard of a row-sharded index plus the merge collective.

    ``index_factory(id_offset)`` builds the local index (default: the HIP ``ItemIndex`` on
    this rank's device). Tests inject a CPU stand-in to run the orchestration under gloo."""

    def __init__(self, n_items: int, *, group=None, device: Optional[int] = None, dtype: str = "f32",
                 index_factory=None):
        import torch.distributed as dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.n = int(n_items)
        self.lo, self.hi = shard_bounds(self.n, self.world, self.rank)
        self.empty = self.hi <= self.lo
        if index_factory is not None:
            self.local = index_factory(self.lo)
        else:
            import torch
            from .engine import ItemIndex
            dev = torch.cuda.current_device() if device is None else device
            self.local = ItemIndex(device=dev, dtype=dtype, id_offset=self.lo)

    # ---------------------------------------------------------------- uploads (own rows only)
    def _mine(self, full_or_shard, axis=0):
        a = full_or_shard
        return a[self.lo:self.hi] if a.shape[axis] == self.n else a

    def upload_items(self, rows, prenormalized: bool = False, present=None):
        """rows: the full [N, d] matrix (each rank keeps its block) or this rank's block."""
        self.d = int(rows.shape[1])
        if self.empty:
            return
        self.local.upload_items(self._mine(rows), prenormalized=prenormalized,
                                present=None if present is None else self._mine(np.asarray(present)))

    def upload_cf(self, factors, present=None):
        if self.empty:
            return
        self.local.upload_cf(self._mine(factors), present=None if present is None else self._mine(np.asarray(present)))

    def upload_attrs(self, num_parts, year, theme_id):
        if self.empty:
            return
        self.local.upload_attrs(self._mine(np.asarray(num_parts)), self._mine(np.asarray(year)),
                                self._mine(np.asarray(theme_id)))

    # ---------------------------------------------------------------- per-rank bitsets
    @property
    def n_local(self) -> int:
        return max(self.hi - self.lo, 0)

    @property
    def words(self) -> int:
        return (self.n_local + 31) // 32

    def mask_bits(self, mask=None, *, pred=None):
        """This rank's item mask as a device bitset (int32 [words]): a ``Predicate`` evaluated
        on the local attribute columns on the device (``bb_eval_mask``), or a global bool [N]
        sliced to this rank's rows once (keep the result and pass it to every ``search``)."""
        import torch
        dev = self._device()
        if self.empty:
            return torch.zeros((0,), dtype=torch.int32, device=dev)
        if pred is not None:
            return self.local.eval_mask_bits(pred)
        from .engine import bits_from_bool
        loc = np.asarray(mask, bool)
        loc = loc[self.lo:self.hi] if loc.shape[0] == self.n else loc
        return torch.as_tensor(bits_from_bool(loc).view(np.int32)).to(dev)

    def excl_bits(self, item_ids):
        """Per-query exclusions (CF: the user's rated sets, recommendation_system.py:441-451) as
        a device bitset [B, words] of this rank's rows, scattered on the device from global item
        ids: a list of B id arrays, or an int64 tensor [B, m] padded with -1.  Ids outside
        [lo, hi) belong to other ranks and are dropped here; repeated ids count once."""
        import torch
        dev = self._device()
        if isinstance(item_ids, torch.Tensor):
            ids = item_ids.to(dev, torch.int64)
            if ids.dim() != 2:
                raise ValueError("excl_bits: an id tensor must be [B, m] (pad with -1)")
            # one bit per distinct id: sort each row and drop repeats (the scatter below adds)
            ids, _ = torch.sort(ids, dim=1)
            rep = torch.zeros_like(ids, dtype=torch.bool)
            rep[:, 1:] = ids[:, 1:] == ids[:, :-1]
            ids = ids.masked_fill(rep, -1)
        else:
            lists = [np.unique(np.asarray(r, np.int64)) for r in item_ids]
            m = max([len(r) for r in lists] + [1])
            pad = np.full((len(lists), m), -1, np.int64)
            for b, r in enumerate(lists):
                pad[b, :len(r)] = r
            ids = torch.from_numpy(pad).to(dev)
        B, W = int(ids.shape[0]), self.words
        flat = torch.zeros((B * max(W, 1),), dtype=torch.int64, device=dev)
        loc = ids - self.lo
        ok = (ids >= 0) & (loc >= 0) & (loc < self.n_local)
        rowi = torch.arange(B, device=dev).unsqueeze(1).expand_as(ids)
        word = (rowi * max(W, 1) + (loc >> 5))[ok]
        flat.index_add_(0, word, torch.ones_like(word) << (loc[ok] & 31))   # distinct ids: sum == or
        flat = (flat + (1 << 31)) % (1 << 32) - (1 << 31)                  # u32 words as int32
        return flat.to(torch.int32).view(B, max(W, 1))[:, :W].contiguous()

    def _local_bits(self, a, rows: bool):
        """A search argument as this rank's device bitset.  Packed words (int32 / uint32, numpy
        or torch) must already be this rank's: shape (words,) for a mask, (B, words) for the
        per-query exclusions — anything else raises (a global or another rank's bitset would
        hand the kernel a buffer of the wrong length).  Bool arrays (global [.., N] or local
        [.., n_local]) are sliced and packed here."""
        import torch
        if a is None:
            return None
        ndim = 2 if rows else 1
        is_t = isinstance(a, torch.Tensor)
        if not is_t:
            a = np.asarray(a)   # lists / tuples of bools or packed words
        if (is_t and a.dtype == torch.bool) or (not is_t and a.dtype == np.bool_):
            from .engine import bits_from_bool
            g = np.asarray(a.cpu() if is_t else a, bool)
            if g.ndim != ndim or g.shape[-1] not in (self.n, self.n_local):
                raise ValueError(f"bool {'exclusions' if rows else 'mask'} must be {ndim}-d over the "
                                 f"{self.n} global or {self.n_local} local items, got {tuple(g.shape)}")
            loc = g[..., self.lo:self.hi] if g.shape[-1] == self.n else g
            return torch.as_tensor(bits_from_bool(loc).view(np.int32)).to(self._device())
        t = a if is_t else torch.from_numpy(np.ascontiguousarray(a))
        if t.dtype not in (torch.int32, torch.uint32) or t.dim() != ndim or t.shape[-1] != self.words:
            raise ValueError(f"packed {'exclusions' if rows else 'mask'} must be int32/uint32 words of this "
                             f"rank's rows, shape {'(B, ' if rows else '('}{self.words}), got {tuple(t.shape)} "
                             f"{t.dtype}")
        if t.dtype == torch.uint32:
            t = t.view(torch.int32)
        return t.to(self._device()).contiguous()

    # ---------------------------------------------------------------- search
    def query_rows(self, item_ids):
        """Rows of global ids, assembled across shards (owner fetch + all-reduce sum)."""
        import torch
        import torch.distributed as dist
        ids = torch.as_tensor(item_ids, dtype=torch.int64)
        if self.empty:
            rows = torch.zeros((int(ids.shape[0]), self.d), dtype=torch.float32, device=self._device())
        else:
            mine = (ids >= self.lo) & (ids < self.hi)
            rows = self.local.get_rows(ids.to(self._device()))
            rows = torch.as_tensor(rows).to(self._device()).float()
            rows[~mine.to(rows.device)] = 0
        dist.all_reduce(rows, group=self.group)
        return rows

    def _device(self):
        import torch
        return getattr(self.local, "torch_device", None) or (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))

    def _local_keys(self, mode, k, q_rows, q_cf, loc_mask, loc_excl, k_side):
        import torch
        if self.empty:   # no rows here: empty lists (key 0) for the gather
            sides, kint = self.local.key_lens(mode, k, k_side)
            B = int((q_rows if q_rows is not None else q_cf).shape[0])
            dev = self._device()
            return (torch.zeros((sides, B, kint), dtype=torch.int64, device=dev),
                    torch.zeros((B,), dtype=torch.int64, device=dev))
        return self.local.search_keys(mode, k, q_rows=q_rows, q_cf=q_cf, mask=loc_mask, excl=loc_excl,
                                      k_side=k_side)

    def search(self, mode: str, k: int, *, q_rows=None, q_items=None, q_cf=None, mask=None, excl=None,
               k_side: int = 0, w_content: float = 0.4, w_cf: float = 0.6, pipeline: int = 1):
        """Global top-k for a replicated batch; every rank returns the same results.
        mask: this rank's device bitset (``mask_bits``: int32 [words]) — or a global bool [N]
        for small cases; excl: this rank's [B, words] device bitset (``excl_bits``) — or a
        global bool [B, N].

        pipeline = c > 1 splits the batch into c query chunks: chunk i's key gather is
        enqueued asynchronously (RCCL's own stream) and overlaps chunk i+1's local search
        (the all-gather overlapped with the last tiles).  Results are identical for
        every c (each query's merge is independent).  Opt-in: each chunk pays the streaming
        search's fixed costs (pilot, candidate selects, launches) again, and no 8-GPU run has
        measured the trade here."""
        import torch
        dev = self._device()
        if mode in ("similar", "hybrid") and q_rows is None:
            q_rows = self.query_rows(q_items)
        loc_mask = self._local_bits(mask, False)
        loc_excl = self._local_bits(excl, True)
        q_rows = None if q_rows is None else torch.as_tensor(q_rows).to(dev).float().contiguous()
        q_cf = None if q_cf is None else torch.as_tensor(q_cf).to(dev).float().contiguous()
        B = int((q_rows if q_rows is not None else q_cf).shape[0])
        c = max(1, min(int(pipeline), B))
        bounds = [(B * i // c, B * (i + 1) // c) for i in range(c)]
        pending = []
        for lo, hi in bounds:
            sl = slice(lo, hi)
            keys, maxk = self._local_keys(mode, k, None if q_rows is None else q_rows[sl],
                                          None if q_cf is None else q_cf[sl], loc_mask,
                                          None if loc_excl is None else loc_excl[sl].contiguous(), k_side)
            pending.append(_gather_lists(keys, maxk, self.group, self.world, async_op=c > 1))
        outs = []
        for finish in pending:
            all_keys, all_max = finish()                                    # [P, sides, b, k_int], [P, b]
            outs.append(self.local.finalize(mode, k, all_keys, all_max, self.world, k_side=k_side,
                                            w_content=w_content, w_cf=w_cf))
        if c == 1:
            return outs[0]
        if isinstance(outs[0][0], torch.Tensor):
            return tuple(torch.cat([o[i] for o in outs], 0) for i in range(3))
        return tuple(np.concatenate([o[i] for o in outs], 0) for i in range(3))
