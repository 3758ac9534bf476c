"""Multi-GPU column sharding of W.

Y[:, n] depends only on TCSC column n, X and b[n], so W's columns split
across ranks with no exchange on the compute path: rank r owns columns
[n0_r, n1_r), holds a rebased TCSC slice and the full X, and produces
Y[:, n0_r:n1_r].  The one collective is the all-gather of those Y column
blocks into the row-major [M, N] result (RCCL over xGMI when the process group
uses the "nccl" backend; gloo on CPU for tests).

Two synthetic-W modes (bench.py):
  * weak  (default): every rank owns N_r columns; W = [W_0 | W_1 | ...] where
    block j is drawn with the generateSparseMatrix law (sparseUtils.h:52-87)
    for K x N_r from block_seed(seed, j).  A rank draws ONLY its own block, so
    setup does not grow with the world size, and rank 0's block is exactly the
    single-GPU workload (block_seed(seed, 0) == seed).  P = 8 with N_r = 16384
    is BASELINE configs[4] (N = 131072).
  * strong: N fixed (configs[2]: 16384) and split N/P per rank; W is drawn
    with the row law over all N columns (tsg_gen_tcsc restricted to the
    rank's columns), so it is the same matrix for every P.

GatherPipeline overlaps the all-gather with compute by M chunks: chunk i+1's
kernel runs while chunk i is gathered (RCCL on its own stream), and the
gathered [P, Mc, w] block is reordered into Y[rows of chunk i, :] by one
strided copy.  One process per GPU (torch.distributed), launched by torchrun.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

import tspgemm as T

_GOLDEN64 = 0x9E3779B97F4A7C15


def column_shard(N: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, near-equal column range of `rank` (first N % world ranks get one more)."""
    base, rem = divmod(N, world)
    n0 = rank * base + min(rank, rem)
    return n0, n0 + base + (1 if rank < rem else 0)


def shard_widths(N: int, world: int) -> List[int]:
    return [b - a for a, b in (column_shard(N, world, r) for r in range(world))]


_MASK64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    """splitmix64's output finaliser (a bijection of 64-bit words)."""
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def block_seed(seed: int, j: int) -> int:
    """Seed of column block j of a weak-scaled W (block 0 keeps `seed`).

    The generator (tsg_gen_tcsc) is a splitmix64 stream whose state advances
    by the golden-ratio constant per draw, so a seed of the form seed + j *
    golden would start block j's stream j draws into block 0's -- nearly the
    same matrix, shifted (tests/test_gpu_configs4.py caught it).  Blocks j > 0
    start from a hashed state instead."""
    if j == 0:
        return int(seed) & _MASK64
    return _mix64((int(seed) + j * 0xD1B54A32D192ED03) & _MASK64)


class ShardedTCSC:
    """This rank's column block of a K x N ternary W, resident on its GPU."""

    def __init__(self, arrays: Sequence[np.ndarray], K: int, N: int, rank: int, world: int,
                 device: int = -1, already_sliced: bool = False):
        self.K, self.N, self.rank, self.world = K, N, rank, world
        self.n0, self.n1 = column_shard(N, world, rank)
        sl = tuple(arrays) if already_sliced else T.tcsc_slice(*arrays, N, self.n0, self.n1)
        self.arrays = sl
        self.local = T.TCSCDevice(*sl, K, self.n1 - self.n0, device=device)
        self.nnz = int(len(sl[2]) + len(sl[3]))

    @classmethod
    def from_tcsc(cls, csp, csn, rip, rin, K, N, rank, world, device=-1) -> "ShardedTCSC":
        return cls((csp, csn, rip, rin), K, N, rank, world, device)

    @staticmethod
    def draw(K: int, N: int, s: int, seed: int, rank: int, world: int, mode: str = "strong"):
        """This rank's TCSC slice of the synthetic W (module docstring), host arrays."""
        n0, n1 = column_shard(N, world, rank)
        if mode == "weak":
            if N % world:
                raise ValueError("weak mode needs N divisible by the world size")
            return T.gen_tcsc(K, n1 - n0, s, block_seed(seed, rank))
        if mode != "strong":
            raise ValueError(f"mode must be 'weak' or 'strong', got {mode!r}")
        return T.gen_tcsc(K, N, s, seed, n0, n1)

    @classmethod
    def generate(cls, K: int, N: int, s: int, seed: int, rank: int, world: int,
                 device: int = -1, mode: str = "strong") -> "ShardedTCSC":
        sl = cls.draw(K, N, s, seed, rank, world, mode)
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
    single strided copy into the row-major output."""
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
    _all_gather_into(gathered, Y_local.contiguous(), group)
    out = torch.empty((M, N), dtype=Y_local.dtype, device=Y_local.device)
    _reorder(gathered.view(world, M, wmax), out, widths)
    return out


class _Done:
    def wait(self):
        return True


def _all_gather_into(out, inp, group=None, async_op: bool = False):
    """all_gather_into_tensor; RCCL ("nccl") gathers device tensors directly.
    A gloo group with device tensors (the multi-rank rehearsal on a one-GPU
    box, scripts/dist_rehearsal.sh) is staged through host memory."""
    import torch.distributed as dist
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        ho = out.new_empty(out.shape, device="cpu")
        dist.all_gather_into_tensor(ho, inp.cpu(), group=group)
        out.copy_(ho)
        return _Done() if async_op else None
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def _reorder(g, out, widths: Sequence[int]) -> None:
    """[P, Mc, wmax] rank-major gather -> row-major out[Mc, N] (one strided copy
    when the widths are equal)."""
    world, Mc, wmax = g.shape
    if all(w == wmax for w in widths):
        out.view(Mc, world, wmax).copy_(g.transpose(0, 1))
        return
    n0 = 0
    for r, w in enumerate(widths):
        out[:, n0:n0 + w].copy_(g[r, :, :w])
        n0 += w


def m_chunks(M: int, chunks: int, align: int = 128) -> List[Tuple[int, int]]:
    """Row ranges of the pipeline: `chunks` near-equal runs, multiples of the
    kernel's 128-row M tile except the last (no partial tiles mid-matrix)."""
    chunks = max(1, min(chunks, (M + align - 1) // align))
    per = ((M + chunks - 1) // chunks + align - 1) // align * align
    out, r = [], 0
    while r < M:
        out.append((r, min(M, r + per)))
        r += per
    return out


class GatherPipeline:
    """Y_full[M, N] = all-gather of every rank's Y[:, n0:n1], overlapped with
    the compute by M chunks (SURVEY.md 8e "overlap the gather with compute by
    chunking M").

        compute(0); ag(0)
        compute(1); ag(1); [side stream: wait(0); reorder(0)]
        ...
        [side stream: wait(C-1); reorder(C-1)]; current stream waits for the side stream

    `compute(r0, r1, Y_chunk)` must enqueue (GPU) or perform (CPU) Y[r0:r1,
    n0:n1] into the contiguous Y_chunk [r1-r0, w_local] on the current stream;
    the all-gather of a chunk is issued async right after its compute, so the
    collective's stream waits for that compute only and runs beside the next
    chunk's kernel.  On the GPU the reorder of a gathered chunk ([P, Mc, w]
    rank-major -> Y_full's rows, one strided copy that moves 2 x 4 Mc N bytes)
    runs on a side stream behind that chunk's collective, beside the next
    chunk's compute (the kernel is VALU-bound, the copy HBM-bound); the
    caller's stream waits for the side stream before run() returns, so the
    whole step stays ordered on it.  Buffers are allocated once: the gather
    buffers in __init__, and for an uneven shard (w_local < the widest shard)
    one contiguous [Mc, w_local] compute buffer per chunk on the first run() --
    no allocation per step."""

    def __init__(self, M: int, N: int, world: int, chunks: int = 4, device=None, dtype=None,
                 group=None):
        import torch
        self.M, self.N, self.world, self.group = M, N, world, group
        self.widths = shard_widths(N, world)
        self.wmax = max(self.widths)
        self.ranges = m_chunks(M, chunks)
        dtype = dtype or torch.float32
        self.Yloc = [torch.zeros((r1 - r0, self.wmax), dtype=dtype, device=device) for r0, r1 in self.ranges]
        self.G = [torch.empty((world * (r1 - r0), self.wmax), dtype=dtype, device=device)
                  for r0, r1 in self.ranges]
        self._narrow = None  # (w_local, [Mc, w_local] buffers) for an uneven shard
        cuda = torch.device(device).type == "cuda" if device is not None else False
        self.side = torch.cuda.Stream(device=device) if cuda else None  # the reorders

    def _narrow_buffers(self, w_local: int):
        if self._narrow is None or self._narrow[0] != w_local:
            self._narrow = (w_local, [Yc.new_empty((Yc.shape[0], w_local)) for Yc in self.Yloc])
        return self._narrow[1]

    def run(self, compute: Callable, Y_full, w_local: int) -> None:
        import torch
        pending = []
        narrow = self._narrow_buffers(w_local) if w_local != self.wmax else None
        main = torch.cuda.current_stream(Y_full.device) if self.side is not None else None
        if main is not None:
            # the side stream's reorders write Y_full and read the gather
            # buffers: ordered after everything the caller enqueued before
            self.side.wait_stream(main)
        for i, (r0, r1) in enumerate(self.ranges):
            Yc = self.Yloc[i]
            if narrow is None:
                compute(r0, r1, Yc)
            else:  # uneven shard: compute contiguous, pad into the gather buffer
                compute(r0, r1, narrow[i])
                Yc[:, :w_local].copy_(narrow[i])
            work = _all_gather_into(self.G[i], Yc, self.group, async_op=True)
            pending.append((i, work))
            if len(pending) > 1:
                self._finish(*pending.pop(0), Y_full)
        for p in pending:
            self._finish(*p, Y_full)
        if main is not None:
            main.wait_stream(self.side)

    def _finish(self, i: int, work, Y_full) -> None:
        import torch
        r0, r1 = self.ranges[i]
        if self.side is None:
            work.wait()
            _reorder(self.G[i].view(self.world, r1 - r0, self.wmax), Y_full[r0:r1], self.widths)
            return
        if isinstance(work, _Done):
            # gloo with device tensors (the one-GPU rehearsal): the gathered
            # chunk was copied in on the caller's stream
            self.side.wait_stream(torch.cuda.current_stream(Y_full.device))
        with torch.cuda.stream(self.side):
            work.wait()  # the side stream waits for the collective (RCCL), not the caller's stream
            _reorder(self.G[i].view(self.world, r1 - r0, self.wmax), Y_full[r0:r1], self.widths)
