"""Multi-GPU column sharding of W.

Y[:, n] depends only on TCSC column n, X and b[n], so W's columns split
across ranks with no exchange on the data path: rank r owns columns
[n0_r, n1_r), holds a rebased TCSC slice (tsg_tcsc_slice) and the full X,
and produces Y[:, n0_r:n1_r].  The only collective is the optional
all-gather of those Y column blocks (RCCL over xGMI when the process group
uses the "nccl" backend; gloo on CPU for tests), followed by one strided
copy from the gathered [world, M, w] layout to row-major [M, N].

One process per GPU (torch.distributed), launched by torchrun.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

import tspgemm as T


def column_shard(N: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, near-equal column range of `rank` (first N % world ranks get one more)."""
    base, rem = divmod(N, world)
    n0 = rank * base + min(rank, rem)
    return n0, n0 + base + (1 if rank < rem else 0)


def shard_widths(N: int, world: int) -> List[int]:
    return [b - a for a, b in (column_shard(N, world, r) for r in range(world))]


class ShardedTCSC:
    """This rank's column block of a K x N ternary W, resident on its GPU."""

    def __init__(self, arrays: Sequence[np.ndarray], K: int, N: int, rank: int, world: int,
                 device: int = -1, already_sliced: bool = False):
        self.K, self.N, self.rank, self.world = K, N, rank, world
        self.n0, self.n1 = column_shard(N, world, rank)
        sl = tuple(arrays) if already_sliced else T.tcsc_slice(*arrays, N, self.n0, self.n1)
        self.local = T.TCSCDevice(*sl, K, self.n1 - self.n0, device=device)
        self.nnz = int(len(sl[2]) + len(sl[3]))

    @classmethod
    def from_tcsc(cls, csp, csn, rip, rin, K, N, rank, world, device=-1) -> "ShardedTCSC":
        return cls((csp, csn, rip, rin), K, N, rank, world, device)

    @classmethod
    def generate(cls, K: int, N: int, s: int, seed: int, rank: int, world: int,
                 device: int = -1) -> "ShardedTCSC":
        """Synthetic W (generateSparseMatrix law); every rank draws the same
        stream and keeps only its columns -- no exchange needed."""
        n0, n1 = column_shard(N, world, rank)
        sl = T.gen_tcsc(K, N, s, seed, n0, n1)
        return cls(sl, K, N, rank, world, device, already_sliced=True)

    def forward(self, X, b_full, Y_local=None):
        """X [M, K] (cuda, fp32, replicated) -> this rank's Y[:, n0:n1]."""
        b = b_full[self.n0:self.n1]
        if not b.is_contiguous():
            b = b.contiguous()
        return self.local.gemm_torch(X, b, Y_local)


def allgather_columns(Y_local, N: int, world: int, group=None):
    """All-gather the Y column blocks of every rank into row-major [M, N].

    Uses all_gather_into_tensor over equal-width (zero-padded) blocks, then a
    single strided copy per rank block into the row-major output."""
    import torch
    import torch.distributed as dist

    M = Y_local.shape[0]
    widths = shard_widths(N, world)
    wmax = max(widths)
    if Y_local.shape[1] != wmax:
        pad = torch.zeros((M, wmax), dtype=Y_local.dtype, device=Y_local.device)
        pad[:, : Y_local.shape[1]] = Y_local
        Y_local = pad
    gathered = torch.empty((world * M, wmax), dtype=Y_local.dtype, device=Y_local.device)
    dist.all_gather_into_tensor(gathered, Y_local.contiguous(), group=group)
    gathered = gathered.view(world, M, wmax)
    out = torch.empty((M, N), dtype=Y_local.dtype, device=Y_local.device)
    n0 = 0
    for r, w in enumerate(widths):
        out[:, n0:n0 + w].copy_(gathered[r, :, :w])
        n0 += w
    return out
