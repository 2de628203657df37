"""Multi-GPU discovery: patient shards per rank, ONE collective per fit.

The discovery regression of ``SINDy.fit`` (reference ``libs_m/ct/src/models/sindy.py:190-192``)
is a sum over patients: G_a = sum_p Theta_p^T Theta_p, b_a = sum_p Theta_p^T xdot_p.  Each rank
owns a contiguous shard of patients, builds its partial (G, b) with the Gram kernel, and a single
all-reduce(SUM) of the packed [A*F*F + A*F] f64 buffer (≈ 900 B for the default library) gives
every rank the global system; STLSQ then runs replicated (bitwise identical on every rank) and
the rollout is embarrassingly parallel over the rank's own patients.  No other data-path
collective exists.  Backend "nccl" is RCCL over xGMI on ROCm; the same code runs on "gloo" for
the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class MomentBuffer:
    """One flat f64 buffer holding the per-arm Gram G[A,F,F] and moments b[A,F], so the
    cross-rank reduction is a single collective."""

    def __init__(self, n_arms: int, n_terms: int, device):
        A, F = int(n_arms), int(n_terms)
        self.n_arms, self.n_terms = A, F
        self.flat = torch.zeros(A * F * F + A * F, dtype=torch.float64, device=device)
        self.G = self.flat[: A * F * F].view(A, F, F)
        self.b = self.flat[A * F * F:].view(A, F)


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced patient shard [lo, hi) of ``rank`` (the first n_total % world ranks
    take one extra patient)."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("invalid shard request")
    q, r = divmod(int(n_total), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def reduce_moments(buf: MomentBuffer, group=None) -> MomentBuffer:
    """Sum the per-rank partial (G, b) over all ranks in place (one all-reduce)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(buf.flat, op=dist.ReduceOp.SUM, group=group)
    return buf


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """Max of a host-measured duration over all ranks (the bench contract's whole-job time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def discover_sharded(x, u, arm, rows, dt, lib, threshold, alpha, buf: MomentBuffer, max_iter=100,
                     unbias=True, fd="smoothed4", workspace=None, group=None, out=None, layout="patient"):
    """Per-rank Gram over the local shard -> one all-reduce -> replicated STLSQ.

    Single rank: the fused ``sindy_fit`` (Gram kernel + finalize/STLSQ in two launches)."""
    from . import ops
    world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
    if out is None:
        A, F = buf.n_arms, buf.n_terms
        out = (torch.empty((A, F), dtype=torch.float64, device=buf.flat.device),
               torch.empty((A, F), dtype=torch.int8, device=buf.flat.device),
               torch.empty((A,), dtype=torch.int32, device=buf.flat.device))
    if world == 1:
        coef, mask, iters, _, _ = ops.sindy_fit(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias,
                                                buf.n_arms, fd, workspace, out=(*out, buf.G, buf.b), layout=layout)
        return coef, mask, iters
    ops.gram(x, u, arm, rows, dt, lib, buf.n_arms, fd, workspace, out=(buf.G, buf.b), layout=layout)
    reduce_moments(buf, group)
    return ops.stlsq(buf.G, buf.b, threshold, alpha, max_iter, unbias, out=out)
