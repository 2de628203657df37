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


class MomentBucket:
    """K consecutive fits' MomentBuffers as views of ONE flat buffer: a stream of fits (the C2 pipeline's
    batch of K steps) reduces all K partial systems with a single collective, paying the all-reduce's
    latency (~10-30 us over xGMI for ~1 KB, latency- not bandwidth-bound) once per K fits."""

    def __init__(self, k: int, n_arms: int, n_terms: int, device):
        A, F = int(n_arms), int(n_terms)
        per = A * F * F + A * F
        self.flat = torch.zeros(int(k) * per, dtype=torch.float64, device=device)
        self.bufs = []
        for q in range(int(k)):
            b = MomentBuffer.__new__(MomentBuffer)
            b.n_arms, b.n_terms = A, F
            b.flat = self.flat[q * per:(q + 1) * per]
            b.G = b.flat[: A * F * F].view(A, F, F)
            b.b = b.flat[A * F * F:].view(A, F)
            self.bufs.append(b)


def reduce_bucket(bucket: MomentBucket, group=None, deterministic: bool = False, force: bool = False,
                  async_op: bool = False):
    """Sum every partial system of the bucket over all ranks in place, in one collective (``force``: issue it
    on a single-rank group too -- the bench's --force-collective measurement of the collective's cost).
    ``async_op``: return the collective's work handle (None when no collective ran); its ``wait()`` makes the
    current stream wait for the result (NCCL/RCCL; gloo blocks the host).  Otherwise the bucket is returned."""
    if _world(group) > 1 or (force and dist.is_available() and dist.is_initialized()):
        if deterministic:
            fixed_order_sum(bucket.flat, group)
        else:
            w = dist.all_reduce(bucket.flat, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
            if async_op:
                return w
    return None if async_op else bucket


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced patient shard [lo, hi) of ``rank`` (the first n_total % world ranks
    take one extra patient)."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("invalid shard request")
    q, r = divmod(int(n_total), int(world))
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def _world(group=None) -> int:
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def fixed_order_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    """Deterministic cross-rank sum in place: all-gather the per-rank buffers and add them in rank
    order on every rank (bitwise reproducible, and equal to a fixed-order CPU sum of the same partials;
    SURVEY.md §5 "deterministic option")."""
    W = _world(group)
    if W > 1:
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t.contiguous(), group=group)
        acc = parts[0].clone()
        for q in parts[1:]:
            acc += q
        t.copy_(acc)
    return t


def reduce_moments(buf: MomentBuffer, group=None, deterministic: bool = False) -> MomentBuffer:
    """Sum the per-rank partial (G, b) over all ranks in place: one all-reduce (RCCL picks ring/tree),
    or with ``deterministic`` one all-gather + rank-ordered sum."""
    if _world(group) > 1:
        if deterministic:
            fixed_order_sum(buf.flat, group)
        else:
            dist.all_reduce(buf.flat, op=dist.ReduceOp.SUM, group=group)
    return buf


def reduce_metric_sums(per_step: torch.Tensor, count: torch.Tensor, last: torch.Tensor | None = None, group=None,
                       deterministic: bool = False):
    """The masked-RMSE partial sums of a rank's shard (``ops.masked_sse``: per-step SSE [T], per-step
    active count [T], last-entry (SSE, count) [2]) summed over ranks in ONE collective of 2T (+2) doubles
    (SURVEY.md §8 E1 "Metrics: all-reduce of (SSE, count)"); predictions stay sharded.  Returns the
    reduced (per_step, count, last)."""
    T = per_step.numel()
    pieces = [per_step.reshape(-1), count.reshape(-1)] + ([last.reshape(-1)] if last is not None else [])
    flat = torch.cat([q.to(torch.float64) for q in pieces])
    if _world(group) > 1:
        if deterministic:
            fixed_order_sum(flat, group)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    out = (flat[:T], flat[T:2 * T])
    return out + ((flat[2 * T:2 * T + 2],) if last is not None else (None,))


def rmse_from_sums(per_step, count, last=None, norm_const: float = 50.0, percentage: bool = True):
    """The reference's metric definitions (time_varying_model.py:236-313) from (reduced) sums: ``orig``
    = sqrt(mean_k(SSE_k / n_k)), ``all`` = sqrt(sum SSE / sum n), ``last`` = sqrt(SSE_last / n_last),
    each / norm_const (x100 as a percentage)."""
    import numpy as np
    per = per_step.detach().cpu().numpy()
    cnt = count.detach().cpu().numpy()
    scale = 100.0 if percentage else 1.0
    with np.errstate(invalid="ignore", divide="ignore"):
        orig = float(np.sqrt((per / cnt).mean()) / norm_const * scale)
        allv = float(np.sqrt(per.sum() / cnt.sum()) / norm_const * scale)
        if last is None:
            return orig, allv
        lh = last.detach().cpu().numpy()
        return orig, allv, float(np.sqrt(lh[0] / lh[1]) / norm_const * scale)


def max_over_ranks(seconds: float, device=None, group=None) -> float:
    """Max of a host-measured duration over all ranks (the bench contract's whole-job time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def discover_sharded(x, u, arm, rows, dt, lib, threshold, alpha, buf: MomentBuffer, max_iter=100,
                     unbias=True, fd="smoothed4", workspace=None, group=None, out=None, layout="patient",
                     deterministic=False):
    """Per-rank Gram over the local shard -> one all-reduce (or, ``deterministic``, the rank-ordered
    all-gather sum) -> replicated STLSQ.  The reference's intended parallel path is the pmap over
    virtual devices at sindy.py:687-699 (dead there, F8); here the shards are real GPUs.

    Single rank: the fused ``sindy_fit`` (Gram kernel + finalize/STLSQ in two launches)."""
    from . import ops
    world = _world(group)
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
    reduce_moments(buf, group, deterministic)
    return ops.stlsq(buf.G, buf.b, threshold, alpha, max_iter, unbias, out=out)


class LaggedSchedule:
    """Bookkeeping of the N > 1 lagged step (``ops.plan_fit_rollout_lagged``, insite_fit_rollout_lagged_f64): one
    launch per step, K fits per all-reduce bucket.  With ``delay`` D (0 or 1), NB = 2 + D buckets rotate and launch k
    (k >= 0):

    * streams cohort k's Gram into partial slot k % 2;
    * (k >= 1) reduces slot (k - 1) % 2 -- cohort k - 1 -- to this rank's G|b at position (k - 1) % K of bucket
      ((k - 1) // K) % NB;
    * (k >= (1 + D) K + 1) solves the STLSQ of cohort c = k - (1 + D) K - 1 from its ALL-REDUCED bucket entry into
      coefficient ring slot c % 3;
    * (k >= (1 + D) K + 2) rolls out cohort k - (1 + D) K - 2 with its ring slot;

    and after launch k with k % K == 0, k >= K, the bucket ((k - 1) // K) % NB (cohorts k - K .. k - 1, complete) is
    all-reduced.  D = 0: on the launch stream, in order (the next launch's solves read it).  D = 1 (round 5): issued
    asynchronously (``all_reduce(async_op=True)``: RCCL's own stream, ordered after the launch) and waited for
    (``wait_before``: the launch stream waits on the collective's completion, the host does not block) only before
    the launch whose solve first reads that bucket, K launches later -- the collective runs beside K launches
    instead of between two of them.  Bucket j is written by launches jK + 1 .. jK + K, reduced after jK + K, read
    by the solves of launches jK + (1 + D) K + 1 .. jK + (2 + D) K and rewritten (as bucket j + NB) from launch
    jK + NB K + 1 on; the solve never reads the bucket its own launch writes, and a coefficient slot is written one
    launch before the rollout that reads it.  Every cohort gets the reference's fit-then-rollout over the WHOLE
    cohort (all ranks' patients), (1 + D) K + 1 launches later than at N = 1."""

    def __init__(self, k: int, delay: int = 0):
        if k < 1:
            raise ValueError("K >= 1 fits per bucket")
        if delay not in (0, 1):
            raise ValueError("delay is 0 (in-order all-reduce) or 1 (overlapped)")
        self.K = int(k)
        self.D = int(delay)
        self.NB = 2 + self.D

    @property
    def lag(self) -> int:
        """Launches between a cohort's Gram and its rollout."""
        return (1 + self.D) * self.K + 2

    def launch(self, k: int) -> dict:
        K, NB, L = self.K, self.NB, (1 + self.D) * self.K
        p = {"gram": k, "slot": k % 2, "reduce": None, "fit": None, "rollout": None, "allreduce_after": None,
             "wait_before": None}
        if k >= 1:
            c = k - 1
            p["reduce"] = (c, (c // K) % NB, c % K)
        if k >= L + 1:
            c = k - L - 1
            p["fit"] = (c, (c // K) % NB, c % K, c % 3)
            if self.D and c % K == 0:     # the first solve from bucket c // K: its all-reduce must be complete
                p["wait_before"] = (c // K) % NB
        if k >= L + 2:
            c = k - L - 2
            p["rollout"] = (c, c % 3)
        if k >= K and k % K == 0:
            p["allreduce_after"] = ((k - 1) // K) % NB
        return p

    def period_of(self) -> int:
        """Launch plans repeat with this period (slots 2, buckets NB K, coefficient ring 3)."""
        import math
        return math.lcm(2, self.NB * self.K, 3)

    @staticmethod
    def period(k: int, delay: int = 0) -> int:
        import math
        return math.lcm(2, (2 + int(delay)) * int(k), 3)
