"""Row-block distributed SpMV: one process per GPU, y assembled by all-gather.

The reference has no multi-device code at all (SURVEY §0, §2 rows "Parallelism
strategies" / "Distributed communication backend"); this is the north_star's
partition: contiguous nnz-balanced row blocks (lhpc_csr_partition_rows), every
rank holding its local CSR block (row_ptr rebased to 0, global column indices)
and a full replica of x; after the local SpMV the y blocks are all-gathered so
y can serve as the next x.  On MI355X the collective is torch.distributed
backend "nccl" = RCCL over xGMI; the same code runs with "gloo" on CPU for the
tests (tests/test_dist.py), where the local product is the oracle.

RCCL's all-gather needs equal counts, so every rank contributes a slice padded
to max_rows; ``assemble`` strips the padding (a no-op for even splits).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np


@dataclass
class RowBlock:
    rank: int
    world: int
    cuts: np.ndarray        # world+1 row cuts
    r0: int
    r1: int
    row_ptr: np.ndarray     # rebased local row_ptr (same dtype as the global one)
    col_idx: np.ndarray     # view into the global arrays
    val: np.ndarray

    @property
    def rows(self) -> int:
        return self.r1 - self.r0

    @property
    def max_rows(self) -> int:
        return int(np.max(np.diff(self.cuts)))


def row_block(row_ptr, col_idx, val, rank: int, world: int) -> RowBlock:
    from . import csr_partition_rows
    cuts = csr_partition_rows(row_ptr, world)
    r0, r1 = int(cuts[rank]), int(cuts[rank + 1])
    k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])
    lrp = (row_ptr[r0:r1 + 1] - row_ptr[r0]).astype(row_ptr.dtype)
    return RowBlock(rank, world, cuts, r0, r1, lrp, col_idx[k0:k1], val[k0:k1])


class DistSpMV:
    """y_full = A·x across ranks.

    ``local_spmv(x, y_out)`` computes this rank's rows into ``y_out`` (a view
    of length ``block.rows``); in production it is a libhpc_amd.SpMVPlan on
    the rank's GPU.  ``step`` = local SpMV + all_gather_into_tensor.
    """

    def __init__(self, block: RowBlock, local_spmv: Callable, like, group=None):
        import torch
        self.block = block
        self.local_spmv = local_spmv
        self.group = group
        m = block.max_rows
        self.y_local = torch.zeros(m, dtype=like.dtype, device=like.device)
        self.y_gather = torch.empty(m * block.world, dtype=like.dtype, device=like.device)

    def step(self, x):
        import torch.distributed as dist
        self.local_spmv(x, self.y_local[:self.block.rows])
        if self.block.world > 1:
            dist.all_gather_into_tensor(self.y_gather, self.y_local, group=self.group)
        else:
            self.y_gather.copy_(self.y_local)
        return self.y_gather

    def assemble(self, out: Optional["object"] = None):
        """Full y (n_rows) from the padded gather buffer."""
        import torch
        b = self.block
        if np.all(np.diff(b.cuts) == b.max_rows):
            return self.y_gather[:int(b.cuts[-1])]
        m = b.max_rows
        parts = [self.y_gather[p * m: p * m + int(b.cuts[p + 1] - b.cuts[p])] for p in range(b.world)]
        return torch.cat(parts) if out is None else torch.cat(parts, out=out)
