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


# --------------------------------------------------------------- stencil7
def slab_bounds(nz: int, rank: int, world: int):
    """Even z-slab split: rank r owns global planes [z0, z1)."""
    base, rem = divmod(nz, world)
    z0 = rank * base + min(rank, rem)
    return z0, z0 + base + (1 if rank < rem else 0)


class DistStencil7:
    """7-point stencil on a z-slab decomposition (BASELINE config C5).

    Every rank holds its slab as HPCHighDimensionFlatArray<3,float,1> of
    logical (nzl, ny, nx): the z ghost planes are halos filled from the
    neighbouring ranks each step (global boundary ranks keep the Dirichlet
    ghost planes they were given).  ``step`` posts the halo send/recv
    (torch.distributed batched P2P — RCCL over xGMI on MI355X), computes the
    interior planes [1, nzl-1) meanwhile, then the two boundary planes.
    ``compute(u, out, z_begin, z_end)`` is the local kernel
    (libhpc_amd.stencil7_planes on the GPU; the oracle in CPU tests).
    """

    def __init__(self, nzl: int, ny: int, nx: int, rank: int, world: int, compute: Callable,
                 group=None):
        self.nzl, self.ny, self.nx = nzl, ny, nx
        self.rank, self.world = rank, world
        self.compute = compute
        self.group = group
        self.plane = (ny + 2) * (nx + 2)

    def _plane(self, t, z):  # padded plane index z in [-1, nzl]
        p = self.plane
        return t[(z + 1) * p:(z + 2) * p]

    def halo_ops(self, u):
        import torch.distributed as dist
        ops = []
        if self.rank > 0:
            ops.append(dist.P2POp(dist.isend, self._plane(u, 0), self.rank - 1, self.group))
            ops.append(dist.P2POp(dist.irecv, self._plane(u, -1), self.rank - 1, self.group))
        if self.rank < self.world - 1:
            ops.append(dist.P2POp(dist.isend, self._plane(u, self.nzl - 1), self.rank + 1, self.group))
            ops.append(dist.P2POp(dist.irecv, self._plane(u, self.nzl), self.rank + 1, self.group))
        return ops

    def step(self, u, out):
        import torch.distributed as dist
        ops = self.halo_ops(u) if self.world > 1 else []
        reqs = dist.batch_isend_irecv(ops) if ops else []
        if self.nzl > 2:
            self.compute(u, out, 1, self.nzl - 1)          # interior: no halo needed
        for r in reqs:
            r.wait()
        self.compute(u, out, 0, min(1, self.nzl))          # boundary planes
        if self.nzl > 1:
            self.compute(u, out, self.nzl - 1, self.nzl)
        return out


# ---------------------------------------------- SpMV with overlapped all-gather
class InterleavedBlocks:
    """Row ownership for overlapped all-gather: the rows are cut into world·K
    blocks; global block b = k·world + r belongs to rank r as its chunk k, so
    the gather of chunk k from every rank is exactly rows
    [cuts[k·world], cuts[(k+1)·world]) of y and each chunk's collective can
    run while the next chunk computes.

    With ``row_ptr`` the cuts are nnz-balanced (binary search on
    row_ptr for the nnz targets, lhpc_csr_partition_rows with world·K parts);
    without it, equal row blocks.  B = the largest block: the torch path pads
    every block to B rows (all_gather needs equal counts) and compacts y; the
    native path (libhpc_amd.DistSpMVPlan) broadcasts exact slices."""

    def __init__(self, n_rows: int, world: int, K: int, row_ptr=None):
        self.n, self.world, self.K = n_rows, world, K
        if row_ptr is not None:
            from . import csr_partition_rows
            self.cuts = csr_partition_rows(row_ptr, world * K).astype(np.int64)
        else:
            b = -(-n_rows // (world * K)) if n_rows else 0
            self.cuts = np.minimum(np.arange(world * K + 1, dtype=np.int64) * b, n_rows)
        self.B = int(np.max(np.diff(self.cuts))) if n_rows else 0
        self.even = bool(np.all(np.diff(self.cuts)[:-1] == self.B)) if n_rows else True

    def rows(self, rank: int, k: int):
        b = k * self.world + rank
        return int(self.cuts[b]), int(self.cuts[b + 1])

    def local_csr(self, row_ptr, col_idx, val, rank: int, k: int):
        r0, r1 = self.rows(rank, k)
        lrp = np.zeros(self.B + 1, dtype=row_ptr.dtype)  # padded to B rows (empty tail rows)
        seg = (row_ptr[r0:r1 + 1] - row_ptr[r0]).astype(row_ptr.dtype)
        lrp[:seg.shape[0]] = seg
        lrp[seg.shape[0]:] = seg[-1]
        k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])
        return lrp, col_idx[k0:k1], val[k0:k1]

    def local_csr_all(self, row_ptr, col_idx, val, rank: int):
        """The rank's K chunks as one CSR of K·B rows (chunk k = rows
        [k·B, (k+1)·B)) and the split rows B, 2B, …, (K−1)·B — the input of
        one row-range plan (SpMVPlan(..., splits=...))."""
        parts = [self.local_csr(row_ptr, col_idx, val, rank, k) for k in range(self.K)]
        lrp = np.zeros(self.K * self.B + 1, dtype=np.int64)
        off = 0
        for k, (prp, _, _) in enumerate(parts):
            lrp[k * self.B:(k + 1) * self.B + 1] = prp.astype(np.int64) + off
            off += int(prp[-1])
        if off < 2 ** 31:
            lrp = lrp.astype(np.int32)
        col = np.concatenate([c for _, c, _ in parts]) if parts else col_idx[:0]
        v = np.concatenate([w for _, _, w in parts]) if parts else val[:0]
        return lrp, col, v, [k * self.B for k in range(1, self.K)]

    def compact_index(self):
        """Positions of y's rows in the padded gather buffer (K·world·B)."""
        idx = np.empty(self.n, dtype=np.int64)
        for b in range(self.world * self.K):
            r0, r1 = int(self.cuts[b]), int(self.cuts[b + 1])
            idx[r0:r1] = b * self.B + np.arange(r1 - r0)
        return idx


class DistSpMVOverlap:
    """y = A·x on `world` ranks, K chunks per rank, all-gather of chunk k
    (async, RCCL stream) overlapped with the SpMV of chunk k+1 — the
    torch.distributed form (any backend; the gloo tests and the 1-GPU
    rehearsal).  The native RCCL form behind the C ABI is
    libhpc_amd.DistSpMVPlan (lhpc_dist_spmv).

    ``local_spmvs[k](x, y_out)`` computes the rank's chunk k (B rows)."""

    def __init__(self, blocks: InterleavedBlocks, local_spmvs, like, group=None):
        import torch
        self.blocks = blocks
        self.fns = local_spmvs
        self.group = group
        B, W, K = blocks.B, blocks.world, blocks.K
        self.y_local = torch.zeros(K, B, dtype=like.dtype, device=like.device)
        self.y_pad = torch.empty(K * W * B, dtype=like.dtype, device=like.device)
        self.idx = None if blocks.even else torch.from_numpy(blocks.compact_index()).to(like.device)
        self.y_full = torch.empty(blocks.n, dtype=like.dtype, device=like.device)

    def step(self, x):
        import torch
        import torch.distributed as dist
        B, W, K = self.blocks.B, self.blocks.world, self.blocks.K
        works = []
        for k in range(K):
            self.fns[k](x, self.y_local[k])
            out = self.y_pad[k * W * B:(k + 1) * W * B]
            if W > 1:
                works.append(dist.all_gather_into_tensor(out, self.y_local[k], group=self.group,
                                                         async_op=True))
            else:
                out.copy_(self.y_local[k])
        for w in works:
            w.wait()
        if self.idx is None:
            return self.y_pad[:self.blocks.n]
        torch.index_select(self.y_pad, 0, self.idx, out=self.y_full)
        return self.y_full


# ------------------------------------------------------------------ CG
class HipOps:
    """CG vector building blocks on the GPU (include/lhpc.h lhpc_vec_dot /
    lhpc_cg_step_xr / lhpc_cg_step_p)."""

    def __init__(self, stream=None):
        self.stream = stream

    def dot(self, a, b, out):
        from . import vec_dot
        vec_dot(a, b, out, stream=self.stream)

    def step_xr(self, num, den, x, p, r, q, rr_out):
        from . import cg_step_xr
        cg_step_xr(num, den, x, p, r, q, rr_out, stream=self.stream)

    def step_p(self, num, den, r, p):
        from . import cg_step_p
        cg_step_p(num, den, r, p, stream=self.stream)

    def step_r(self, num, den, r, q, rr_out):
        from . import cg_step_r
        cg_step_r(num, den, r, q, rr_out, stream=self.stream)

    def step_xp(self, anum, aden, bnum, bden, x, p, r):
        from . import cg_step_xp
        cg_step_xp(anum, aden, bnum, bden, x, p, r, stream=self.stream)


class TorchCPUOps:
    """The same building blocks on CPU tensors — for the gloo tests of the
    distributed control flow only (the GPU path uses HipOps)."""

    def dot(self, a, b, out):
        import torch
        out.copy_(torch.dot(a.double(), b.double()).reshape(1))

    def step_xr(self, num, den, x, p, r, q, rr_out):
        a = (num / den).to(x.dtype)
        x.add_(a * p)
        r.sub_(a * q)
        self.dot(r, r, rr_out)

    def step_p(self, num, den, r, p):
        beta = (num / den).to(p.dtype)
        p.mul_(beta).add_(r)

    def step_r(self, num, den, r, q, rr_out):
        a = (num / den).to(r.dtype)
        r.sub_(a * q)
        self.dot(r, r, rr_out)

    def step_xp(self, anum, aden, bnum, bden, x, p, r):
        a = (anum / aden).to(x.dtype)
        x.add_(a * p)
        if bnum is not None:
            self.step_p(bnum, bden, r, p)


class DistCG:
    """Conjugate gradient on `world` ranks (one per GPU): contiguous equal row
    blocks (InterleavedBlocks(n, world, 1)), every rank holding its block of
    A (an SpMVPlan over the global columns), its blocks of x, r, q and a full
    replica of p.  Per iteration: local q = A_blk·p; p·q and r·r are
    all-reduced (RCCL over xGMI with backend "nccl"); after p = r + β·p the
    p blocks are all-gathered so the next SpMV sees the whole p — the
    "y becomes the next x" exchange of SURVEY §8e/§8f.  Padding rows (block
    size × world > n) are empty rows with b = 0, so they stay 0 and do not
    touch the dots.

    ``local_spmv(p_full_n, q_block)`` computes this rank's block;
    ``local_spmv_dot(p_full_n, q_block, w_block, out)``, if given, also
    writes w·q into ``out`` in the same pass (lhpc_spmv_dot: the p·q dot
    fused into the ADAPTIVE epilogue);
    ``ops``: HipOps (GPU) or TorchCPUOps (gloo tests)."""

    def __init__(self, blocks: InterleavedBlocks, rank: int, local_spmv: Callable, ops, like, group=None,
                 local_spmv_dot: Optional[Callable] = None):
        import torch
        assert blocks.K == 1
        self.blocks, self.rank, self.fn, self.ops, self.group = blocks, rank, local_spmv, ops, group
        self.fn_dot = local_spmv_dot
        B, W = blocks.B, blocks.world
        self.p_full = torch.zeros(B * W, dtype=like.dtype, device=like.device)
        # world 1: p is the replica itself (no gather copy)
        self.p = self.p_full[:B] if W == 1 else torch.zeros(B, dtype=like.dtype, device=like.device)
        self.r = torch.zeros_like(self.p)
        self.q = torch.zeros_like(self.p)
        self.s = torch.zeros(4, dtype=torch.float64, device=like.device)  # rr0, rr1, pq, bb

    def _allreduce(self, t):
        import torch.distributed as dist
        if self.blocks.world > 1:
            dist.all_reduce(t, group=self.group)

    def _gather(self, dst, src):
        import torch.distributed as dist
        if self.blocks.world > 1:
            dist.all_gather_into_tensor(dst, src, group=self.group)
        elif dst.data_ptr() != src.data_ptr():
            dst[:src.numel()].copy_(src)

    def solve(self, b, x, tol: float = 1e-8, max_iter: int = 1000, check_every: int = 1):
        """b, x: this rank's blocks (length B, padded rows 0); x updated in
        place.  Returns (x, iterations, ‖r‖/‖b‖)."""
        n = self.blocks.n
        s = self.s
        rr = [s[0:1], s[1:2]]
        pq, bb = s[2:3], s[3:4]
        self.ops.dot(b, b, bb)
        self._allreduce(bb)
        self._gather(self.p_full, x)          # x_full for r = b − A·x
        self.fn(self.p_full[:n], self.q)
        self.r.copy_(b)
        self.r.sub_(self.q)
        self.p.copy_(self.r)
        self.ops.dot(self.r, self.r, rr[0])
        self._allreduce(rr[0])
        h_bb = float(bb.item())
        stop = tol * tol * (h_bb if h_bb > 0 else 1.0)
        h_rr = float(rr[0].item())
        cur, it = 0, 0
        if h_rr > stop:
            self._gather(self.p_full, self.p)
            for it in range(1, max_iter + 1):
                if self.fn_dot is not None:
                    self.fn_dot(self.p_full[:n], self.q, self.p, pq)
                else:
                    self.fn(self.p_full[:n], self.q)
                    self.ops.dot(self.p, self.q, pq)
                self._allreduce(pq)
                # r -= α·q, rr' = r·r; the x update rides with the p update
                # (one vector pass less; lhpc_cg_step_r / lhpc_cg_step_xp)
                self.ops.step_r(rr[cur], pq, self.r, self.q, rr[cur ^ 1])
                self._allreduce(rr[cur ^ 1])
                if it % check_every == 0 or it == max_iter:
                    h_rr = float(rr[cur ^ 1].item())
                    if not np.isfinite(h_rr):
                        raise FloatingPointError("DistCG: breakdown (non-finite residual)")
                    if h_rr <= stop:
                        self.ops.step_xp(rr[cur], pq, None, None, x, self.p, None)
                        break
                self.ops.step_xp(rr[cur], pq, rr[cur ^ 1], rr[cur], x, self.p, self.r)
                self._gather(self.p_full, self.p)
                cur ^= 1
        res = float(np.sqrt(max(h_rr, 0.0)) / np.sqrt(h_bb if h_bb > 0 else 1.0))
        return x, it, res
