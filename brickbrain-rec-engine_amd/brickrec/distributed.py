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

At 25K items the index does not shard (39 MB); ``bench.py --gpus N`` runs replicas.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def _all_gather(t, group, world):
    """Gather equal-shape tensors -> [world, *t.shape] (one buffer with nccl/RCCL)."""
    import torch
    import torch.distributed as dist
    out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    else:
        dist.all_gather(list(out.unbind(0)), t.contiguous(), group=group)
    return out


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

    def search(self, mode: str, k: int, *, q_rows=None, q_items=None, q_cf=None, mask=None, excl=None,
               k_side: int = 0, w_content: float = 0.4, w_cf: float = 0.6):
        """Global top-k for a replicated batch; every rank returns the same results.
        mask: global bool [N] (or None); excl: global bool [B, N] (or None)."""
        import torch
        dev = self._device()
        if mode in ("similar", "hybrid") and q_rows is None:
            q_rows = self.query_rows(q_items)
        loc_mask = None if mask is None else torch.as_tensor(np.asarray(mask)[self.lo:self.hi])
        loc_excl = None if excl is None else torch.as_tensor(np.asarray(excl)[:, self.lo:self.hi])
        from .engine import bits_from_bool
        if loc_mask is not None:
            loc_mask = torch.as_tensor(bits_from_bool(loc_mask.numpy()).view(np.int32)).to(dev)
        if loc_excl is not None:
            loc_excl = torch.as_tensor(bits_from_bool(loc_excl.numpy()).view(np.int32)).to(dev)
        q_rows = None if q_rows is None else torch.as_tensor(q_rows).to(dev).float().contiguous()
        q_cf = None if q_cf is None else torch.as_tensor(q_cf).to(dev).float().contiguous()
        if self.empty:   # no rows here: empty lists (key 0) for the gather
            sides, kint = self.local.key_lens(mode, k, k_side)
            B = int((q_rows if q_rows is not None else q_cf).shape[0])
            keys = torch.zeros((sides, B, kint), dtype=torch.int64, device=dev)
            maxk = torch.zeros((B,), dtype=torch.int64, device=dev)
        else:
            keys, maxk = self.local.search_keys(mode, k, q_rows=q_rows, q_cf=q_cf, mask=loc_mask,
                                                excl=loc_excl, k_side=k_side)
        all_keys = _all_gather(keys, self.group, self.world)   # [P, sides, B, k_int]
        all_max = _all_gather(maxk, self.group, self.world)    # [P, B]
        return self.local.finalize(mode, k, all_keys, all_max, self.world, k_side=k_side,
                                   w_content=w_content, w_cf=w_cf)
