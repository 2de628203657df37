#!/usr/bin/env python3
"""Headline benchmark: patient-trajectories/s of the INSITE hot path on MI355X.

One "step" = one pass of the hot path over one synthetic batch (BASELINE.json configs[1], C2):
    discovery  — fused savgol(5,3) + 4th-order FD + poly2 library + per-arm Gram   (gram kernel)
               — [N>1: one RCCL all_reduce(SUM) of the 2 x (49 + 7) Gram/moment doubles]
               — STLSQ(threshold 0.1, alpha 0.5) + unbias                          (stlsq kernel)
    rollout    — RK4 counterfactual rollout of every patient over T steps          (rollout kernel)
on N_per_gpu = 100,000 patients x T = 200 steps, fp64, inputs resident in HBM (generated on
device before timing).  Weak scaling: every rank holds its own 100k-patient shard.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")
sys.path.insert(0, PKG_DIR)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "patient-trajectories/sec (N×T RK4 steps) at 1/2/4/8 GPUs; RMSE vs CPU ref"
HBM_PEAK_GBPS = 8000.0     # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)


# Untimed warmup steps when --warmup is not given.  The C5 rollout reaches its steady state only after a few dozen
# calls (5 warmup steps: 0.79 ms/step by the wall clock while the per-launch events already read 0.73; 60: 0.71 and
# 0.715 agree), C4 and F4 after a few hundred of their short steps (5 %), the C3 Gram's launches 0.8 % after 20
# (8.15 -> 8.08 ms); C2 and INSITE do not move (profiles/r05/warm/).  Warmup is outside the timed region either way
# and the line reports the count used.
WARMUP_DEFAULT = {"c5": 60, "c4": 200, "f4": 200, "c3": 20}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warmup steps (default: 5; C5 60, C4 / F4 200, C3 20 -- see WARMUP_DEFAULT)")
    ap.add_argument("--rk45-identity-order", action="store_true",
                    help="C5 ablation: lane r runs row r (no binning by n_obs)")
    ap.add_argument("--rk45-bin", default="attempts", choices=["nobs", "attempts"],
                    help="C5 lane binning key: the per-patient attempt counts the previous step left (default: a C5 "
                         "step re-rolls the same cohort, so waves group equal attempt counts; VERDICT r05 item 7: "
                         "0.660 vs 0.707 ms/step, profiles/r06/c5_bin/) or n_obs (the number of observation intervals)")
    ap.add_argument("--patients", type=int, default=100_000, help="patients per GPU (C2: 100k)")
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--method", default="rk4", choices=["rk4", "euler5"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--layout", default="time", choices=["time", "patient"],
                    help="HBM layout of the per-step arrays (DESIGN.md): time-major is the fast path")
    ap.add_argument("--arm-format", default="bits", choices=["bits", "tiles", "int8"],
                    help="per-step arms of the time-major rollout: 1-bit mask (A <= 2) in time-major rows, the same "
                         "bits tile-major (ops.tile_major_bits: a tile's 32-step group in 256 contiguous bytes), or int8")
    ap.add_argument("--ns-arms", default="tiles", choices=["bits", "tiles"],
                    help="bit-arm layout of the north-star blocks (1M x 500): time-major rows or tile-major "
                         "(default: at 1M patients the time-major rows' 128-B lines, 16 tiles each, leave the L2 "
                         "between their tiles' waves -- profiles/r06/tiles/)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default=None, choices=["deferred", "lagged", "fused", "graph", "seq", "pipeline"],
                    help="deferred (default at N = 1) / fused: ONE launch per step -- the discovery of step i and "
                         "the rollout of step i-1 in the same launch; deferred: the same with the discovery's "
                         "reduction + STLSQ moved into the next launch (step_deferred_kernel); lagged (default at "
                         "N > 1, where the RCCL all-reduce sits between the gram and STLSQ): the deferred kernel with "
                         "the reduction and the STLSQ in separate roles, one all-reduce per --pipe-k launches on the "
                         "launch stream; pipeline: discovery | rollout on two streams, "
                         "consecutive steps overlapped; seq: eager launches on one stream; graph: the seq step in a "
                         "HIP graph")
    ap.add_argument("--stlsq-stream", default="discovery", choices=["discovery", "rollout"],
                    help="pipeline mode, N = 1: run each step's STLSQ in the gram's last block on the discovery "
                         "stream (default) or as its own launch on the rollout stream ahead of that step's rollout "
                         "(off the discovery stream's critical path)")
    ap.add_argument("--dstreams", type=int, default=1,
                    help="deferred mode: independent streams of cohorts, launch k on stream k %% S (1 = one stream)")
    ap.add_argument("--pipe-k", type=int, default=4, help="pipeline: steps per batch (one event per batch per stream)")
    ap.add_argument("--lag-k", type=int, default=16,
                    help="lagged mode: fits per all-reduce bucket (profiles/r05/lagk: at N = 1 with the single-rank RCCL "
                         "collective, K = 4 / 8 / 16 all within 1.2-2 %% of the deferred step)")
    ap.add_argument("--lag-delay", type=int, default=1, choices=[0, 1],
                    help="lagged mode: 0 = the bucket all-reduce in order on the launch stream, 1 = issued async and "
                         "waited for K launches later (insite_amd.dist.LaggedSchedule delay; at K = 16 as cheap as 0 "
                         "at N = 1, and the N > 1 collective's latency runs beside K launches)")
    ap.add_argument("--pipe-rs", type=int, default=2, help="pipeline: rollout streams taking alternate batches")
    ap.add_argument("--fused-graph", action="store_true",
                    help="fused mode: replay the ping-pong pair of step launches from a HIP graph")
    ap.add_argument("--no-fused", action="store_true",
                    help="pipeline mode at N = 1: skip the secondary fused-step measurement")
    ap.add_argument("--gram-blocks", type=int, default=0,
                    help="fused mode: blocks of the step kernel's resident round given to the discovery (0 = the "
                         "library's default split)")
    ap.add_argument("--cpu-sample", type=int, default=100_000, help="patients in the timed CPU sample")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the north-star blocks of the C2 line: the 1M x 500 rollout roofline probe and the full "
                         "1M x 500 deferred step (discovery + RK4 rollout, north_star_step)")
    ap.add_argument("--ns-steps", type=int, default=10, help="timed launches of the north_star_step block")
    ap.add_argument("--no-c3-block", action="store_true",
                    help="skip the compact C3 block (BASELINE configs[2], the largest single-GPU configuration) of "
                         "the default C2 line")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle check of the benched cohort (every line: a sample of the last timed step's "
                         "rows through the oracle after the timed region)")
    ap.add_argument("--force-collective", action="store_true",
                    help="C2 at N = 1: join a single-rank RCCL process group and run the N > 1 pipeline's data path "
                         "(gram, one bucketed all_reduce per batch, STLSQ) so the collective and the process "
                         "group's stream synchronisation sit in the timed region")
    ap.add_argument("--no-rotate", action="store_true",
                    help="C2 fused: one cohort re-read every step (default: two cohorts alternate, so no step "
                         "re-reads data the 256 MB Infinity Cache still holds)")
    ap.add_argument("--isolated", action="store_true",
                    help="also time each C2 kernel in isolation (back-to-back launches on one stream)")
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "insite", "insite4", "f4", "ns"],
                    help="c2: BASELINE configs[1], the headline line (default); c3: configs[2], the 5-state fp32 "
                         "system (parity-test configuration, measured separately)")
    ap.add_argument("--insite-order", default="nfev", choices=["seq_len", "nfev"],
                    help="insite line: lanes binned by the row's window (seq_len) or by window and the previous "
                         "step's evaluation counts (nfev)")
    ap.add_argument("--insite-only-binned", action="store_true",
                    help="--config insite: time only the product route (skip the identity-order and prepare-route "
                         "comparisons; for counter runs)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r02.json"),
                    help="per-launch HBM bytes from the rocprofv3 PMC passes (profiles/), if present")
    args = ap.parse_args()
    if args.warmup is None:
        args.warmup = WARMUP_DEFAULT.get(args.config, 5)
    return args


class HipEvents:
    """hipEventRecord / hipStreamWaitEvent on raw handles (the HIP runtime torch already loaded)."""

    def __init__(self):
        import ctypes
        self._c = ctypes
        self._hip = ctypes.CDLL("libamdhip64.so.7")
        self._hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        self._hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self._hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self._hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self._events = []

    def create(self, timing=False):
        e = self._c.c_void_p()
        # ordering events: hipEventDisableTiming | hipEventReleaseToDevice -- the consumers are queues of
        # this device, so a device-scope release suffices; the default system-scope release writes back
        # and invalidates the caches at every record (~20 us of dead queue time per step on ROCm 7.2:
        # profiles/r02/c2_pipeline_trace.txt)
        flags = 0x0 if timing else (0x2 | 0x40000000)
        if self._hip.hipEventCreateWithFlags(self._c.byref(e), flags) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")
        self._events.append(e)
        return e

    def elapsed_ms(self, e0, e1):
        ms = self._c.c_float()
        if self._hip.hipEventElapsedTime(self._c.byref(ms), e0, e1) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def record(self, e, stream):
        if self._hip.hipEventRecord(e, self._c.c_void_p(stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def wait(self, stream, e):
        if self._hip.hipStreamWaitEvent(self._c.c_void_p(stream), e, 0) != 0:
            raise RuntimeError("hipStreamWaitEvent failed")

    def __del__(self):
        for e in getattr(self, "_events", []):
            self._hip.hipEventDestroy(e)


def bits_layout(fmt):
    """counterfactual_arms layout of a bit-arm format name (--arm-format / --ns-arms)."""
    return "tile_bits" if fmt == "tiles" else "time_bits"


def rollout_bytes(N, T, U=2, w=8, arm_bits=8):
    """Algorithmic HBM bytes of one rollout launch:
    N*T*(S*w + arm_bits/8) [state out + per-step arm in: int8 = 8 bits, packed = 1 bit]
    + N*(S*w + U*w) [y0 + statics in]."""
    return N * T * w + (N * T * arm_bits + 7) // 8 + N * (w + U * w)


def gram_bytes(N, L, U=2, w=8):
    """Algorithmic HBM bytes of one discovery pass: the L = T observations of every patient
    (x[p, 0..L-1] feed the L-1 rows' smoothing stencils) + statics, arm byte and row count."""
    return N * L * w + N * (U * w + 1 + 4)


# --------------------------------------------------------------------------------------------------
# CPU baseline: the oracle's numpy restatement on every worker the host grants this
# job, plus the scipy.integrate.solve_ivp(RK45) leg the north star names.  Run on rank 0 at N = 1,
# BEFORE the GPU is initialised (the worker pool forks a GPU-free process).
# --------------------------------------------------------------------------------------------------
def host_info():
    """CPU model, os.cpu_count(), the affinity mask and the worker count used."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    # the box grants a CPU share (OMP_NUM_THREADS is set to it there); os.cpu_count() is the machine
    share = os.environ.get("INSITE_CPU_WORKERS") or os.environ.get("OMP_NUM_THREADS")
    workers = max(1, min(aff, int(share))) if share else aff
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "sched_affinity": aff, "workers": workers}


@contextlib.contextmanager
def worker_pool(ctx, W, initializer, initargs=()):
    """A process pool that ends with close() + join(): the workers exit on their own once the work is done.  (The
    Pool context manager's terminate() SIGTERMs them, which under rocprofv3 -- whose preloaded library the workers
    inherit -- printed an "Aborted at" stack per worker into every profiler log)"""
    pool = ctx.Pool(W, initializer=initializer, initargs=initargs)
    try:
        yield pool
    except BaseException:
        pool.terminate()
        pool.join()
        raise
    pool.close()
    pool.join()


_CPU = {}


def _cpu_worker_init():
    """One BLAS thread per worker process (the pool supplies the parallelism)."""
    try:
        from threadpoolctl import threadpool_limits
        _CPU["limiter"] = threadpool_limits(limits=1)
    except Exception:  # pragma: no cover
        pass


def _cpu_gram_chunk(bounds):
    from oracle import insite_ref as R
    lo, hi = bounds
    d = _CPU
    return R.gram_moments_vectorized(d["x"][lo:hi], d["u"][lo:hi], d["arm"][lo:hi], d["T"] - 2, d["dt"], d["exps"])


def _cpu_rollout_chunk(bounds):
    from oracle import insite_ref as R
    lo, hi = bounds
    d = _CPU
    y = R.rollout(d["x"][lo:hi, 0], d["u"][lo:hi], d["arms"][lo:hi], d["coef"], d["exps"], d["dt"], method=d["method"])
    return float(y[:, -1].sum())


def _cpu_ivp_chunk(bounds):
    """scipy.integrate.solve_ivp(RK45, rtol = atol = 1.4e-8) per patient over the whole horizon with the
    piecewise-constant per-step arm, t_eval on the observation grid and max_step = dt/10 — the
    reference's own call pattern (utils/exp_utils.py:140)."""
    from scipy.integrate import solve_ivp
    lo, hi = bounds
    d = _CPU
    T, dt, coef, exps = d["T"], d["dt"], d["coef"], d["exps"]
    grid = np.arange(1, T + 1) * dt
    acc = 0.0
    for p in range(lo, hi):
        u = d["u"][p]
        arms = d["arms"][p]
        mono = np.array([np.prod([u[i - 1] ** e[i] for i in range(1, e.size)]) for e in exps])
        al = np.array([sum(coef[a, j] * mono[j] for j in range(exps.shape[0]) if exps[j, 0] == 0 and abs(coef[a, j]) > 1e-3)
                       for a in range(coef.shape[0])])
        be = np.array([sum(coef[a, j] * mono[j] for j in range(exps.shape[0]) if exps[j, 0] == 1 and abs(coef[a, j]) > 1e-3)
                       for a in range(coef.shape[0])])

        def f(t, y):
            a = arms[min(int(t / dt), T - 1)]
            return al[a] + be[a] * y
        sol = solve_ivp(f, (0.0, T * dt), [d["x"][p, 0]], method="RK45", t_eval=grid, rtol=1.4e-8, atol=1.4e-8,
                        max_step=dt / 10.0)
        acc += float(sol.y[0, -1])
    return acc


def cpu_baseline(n_sample, T, method, seed, ivp_per_worker=100):
    """Bounded CPU sample of the C2 workload (EQ_4_C cohort, T steps) on the host's workers:
    (1) the oracle's numpy restatement, patients chunked over a process pool (partial Grams summed,
        STLSQ, chunked rollout) — ``value``;
    (2) scipy.integrate.solve_ivp(RK45, rtol = atol = 1.4e-8) per patient (the rollout only) on
        ``ivp_per_worker`` patients per worker, extrapolated linearly — ``scipy_solve_ivp``."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    info = host_info()
    W = info["workers"]
    rng = np.random.default_rng(seed)
    p = R.draw_params(n_sample, "EQ_4_C", rng)
    sim = R.simulate_factual(p, T, rng, "EQ_4_C", 2.0)
    arm = sim["treatment_application"][:, 0].astype(np.int64)
    flip = rng.integers(0, T, size=(n_sample, 1))
    _CPU.update(x=sim["cancer_volume"], u=np.stack([sim["observed_static_c_0"], sim["observed_static_c_1"]], axis=1),
                arm=arm, arms=np.where(np.arange(T)[None, :] >= flip, 1 - arm[:, None], arm[:, None]),
                exps=R.poly_library(3, 2, True), dt=R.MAX_TIME_HORIZON / T, T=T, method=method)
    chunks = [(int(a[0]), int(a[-1]) + 1) for a in np.array_split(np.arange(n_sample), W) if a.size]
    ctx = mp.get_context("fork")          # no GPU context exists yet in this process
    with worker_pool(ctx, W, _cpu_worker_init) as pool:
        pool.map(abs, range(W))           # workers up before the clock starts
        t0 = time.perf_counter()
        parts = pool.map(_cpu_gram_chunk, chunks)
        G = sum(q[0] for q in parts)
        b = sum(q[1] for q in parts)
        _CPU["coef"] = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
        el_disc = time.perf_counter() - t0
    with worker_pool(ctx, W, _cpu_worker_init) as pool:   # forked after the fit: workers see the coefficients
        pool.map(abs, range(W))
        t1 = time.perf_counter()
        pool.map(_cpu_rollout_chunk, chunks)
        el_roll = time.perf_counter() - t1
        n_ivp = min(n_sample, ivp_per_worker * W)
        ivp_chunks = [(int(a[0]), int(a[-1]) + 1) for a in np.array_split(np.arange(n_ivp), W) if a.size]
        t2 = time.perf_counter()
        pool.map(_cpu_ivp_chunk, ivp_chunks)
        el_ivp = time.perf_counter() - t2
    total = el_disc + el_roll
    return {"value": n_sample / total, "unit": "patient-trajectories/s", "cores": W, "kind": "port",
            "sample": f"oracle/insite_ref.py numpy fp64 over a {W}-process pool: {n_sample} EQ_4_C patients x {T} "
                      f"steps, discovery (chunked Gram + STLSQ) {el_disc:.2f} s + {method} rollout {el_roll:.2f} s",
            "host": info,
            "scipy_solve_ivp": {
                "value": n_ivp / el_ivp, "unit": "patient-trajectories/s (rollout only)", "cores": W,
                "kind": "scipy.integrate.solve_ivp(method='RK45', rtol=atol=1.4e-8, max_step=dt/10, t_eval=grid)",
                "sample": f"{n_ivp} patients x {T} steps on {W} workers in {el_ivp:.2f} s; the rate extrapolates "
                          f"linearly in patients (independent solves); {n_sample} patients would take "
                          f"{el_ivp * n_sample / n_ivp:.1f} s"}}


def _cpu_c3_gen(job):
    from oracle import multistate_ref as M
    lo, hi, T, seed = job
    x, a = M.c3_cohort(hi - lo, T, seed=seed)
    a_cf = M.treatment_markov(hi - lo, T, np.random.default_rng(seed + 17))
    return x, a, a_cf


def _cpu_c3_gram_chunk(bounds):
    from oracle import multistate_ref as M
    lo, hi = bounds
    d = _CPU
    return M.ms_gram_vectorized(d["x"][lo:hi], d["a"][lo:hi], M.DT_C3, d["exps"])


def _cpu_c3_rollout_chunk(bounds):
    from oracle import multistate_ref as M
    lo, hi = bounds
    d = _CPU
    y = M.ms_rollout(d["x"][lo:hi, 0].astype(np.float64), d["a_cf"][lo:hi], d["coef"], d["exps"], M.DT_C3, "rk4")
    return float(y[:, -1].sum())


def c3_cpu_baseline(per_worker, T, seed):
    """Bounded CPU sample of the C3 workload (oracle/multistate_ref.py, numpy fp64) on the host's workers:
    discovery (vectorised S-state Gram per chunk, partials summed, one STLSQ per state) + RK4 rollout under
    a fresh Markov treatment sequence — the same step the GPU line times.  The cohort is generated by the
    same pool before the clock starts."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import multistate_ref as M
    info = host_info()
    W = info["workers"]
    n = per_worker * W
    ctx = mp.get_context("fork")
    with worker_pool(ctx, W, _cpu_worker_init) as pool:
        parts = pool.map(_cpu_c3_gen, [(w * per_worker, (w + 1) * per_worker, T, seed + 101 * w) for w in range(W)])
    _CPU.update(x=np.concatenate([p[0] for p in parts]), a=np.concatenate([p[1] for p in parts]),
                a_cf=np.concatenate([p[2] for p in parts]), exps=M.c3_library())
    del parts
    chunks = [(w * per_worker, (w + 1) * per_worker) for w in range(W)]
    with worker_pool(ctx, W, _cpu_worker_init) as pool:
        pool.map(abs, range(W))
        t0 = time.perf_counter()
        gb = pool.map(_cpu_c3_gram_chunk, chunks)
        G = sum(q[0] for q in gb)
        B = sum(q[1] for q in gb)
        _CPU["coef"] = M.ms_stlsq(G, B)[0]
        el_disc = time.perf_counter() - t0
    with worker_pool(ctx, W, _cpu_worker_init) as pool:   # forked after the fit: workers see the model
        pool.map(abs, range(W))
        t1 = time.perf_counter()
        pool.map(_cpu_c3_rollout_chunk, chunks)
        el_roll = time.perf_counter() - t1
    truth = M.c3_truth_coef(_CPU["exps"])
    support_ok = bool(np.array_equal(np.abs(_CPU["coef"]) > 0, truth != 0))
    for k in ("x", "a", "a_cf", "coef"):
        _CPU.pop(k, None)
    return {"value": n / (el_disc + el_roll), "unit": "patient-trajectories/s", "cores": W, "kind": "port",
            "sample": f"oracle/multistate_ref.py numpy fp64 over a {W}-process pool: {n} C3 patients x {T} steps, "
                      f"discovery (chunked S-state Gram + STLSQ per state) {el_disc:.2f} s + RK4 rollout "
                      f"{el_roll:.2f} s; support equals truth: {support_ok}",
            "host": info}


def c3_main(args):
    """Configuration C3 (BASELINE.json configs[2]): 5-state coupled ODE + binary per-step treatment,
    1M patients x 500 steps, fp32 storage, fp64 Gram on MFMA.  One step = discovery (gram_ms on f64
    MFMA + fixed-order finalize + one wave-STLSQ per state) + RK4 counterfactual rollout of every
    patient under a fresh treatment sequence.  Single GPU (patients would shard like C2)."""
    N = args.patients if args.patients != 100_000 else 1_000_000
    T = args.T if args.T != 200 else 500
    cpu = None
    if os.environ.get("WORLD_SIZE", "1") == "1" and not args.no_cpu_baseline:
        # 2000 patients per worker (~0.8 s of discovery + rollout each; the cohort build is untimed)
        cpu = c3_cpu_baseline(max(64, min(2000, args.cpu_sample // 50)), T, args.seed + 3)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = c3_measure(args, dev, N, T, args.steps, args.warmup, not args.no_parity)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    emit(out)


def c3_measure(args, dev, N, T, steps, warmup, parity=True):
    """The C3 line's measurement (c3_main; also the compact ``c3`` block of the default C2 line):
    ``steps`` timed discovery + rollout steps after ``warmup``, per-kernel HIP-event averages, the oracle parity."""
    from insite_amd import multistate as MS
    coh = MS.synthetic_c3(N, T, seed=args.seed, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 17)
    a_cf = MS.markov_treatment_bits(N, T, g, dev)
    lib = coh.lib
    F, S = lib.n_terms, lib.n_states
    G = torch.empty((F, F), dtype=torch.float64, device=dev)
    B = torch.empty((F, S), dtype=torch.float64, device=dev)
    coef = torch.empty((S, F), dtype=torch.float64, device=dev)
    mask = torch.empty((S, F), dtype=torch.int8, device=dev)
    iters = torch.empty((S,), dtype=torch.int32, device=dev)
    y = torch.empty((T, S, N), dtype=torch.float32, device=dev)

    def disc():
        MS.gram_ms(coh.x, coh.a, lib, coh.dt, out=(G, B))
        MS.stlsq_wave(G, B, MS.THRESHOLD_C3, MS.ALPHA_C3, out=(coef, mask, iters))

    # the rollout is specialised (hipRTC, once) to the support the discovery returns; every launch
    # re-checks the device coefficients against it and takes the dense RHS if a term falls outside
    support = [None]

    def roll():
        MS.rollout_ms(coh.y0, a_cf, coef, lib, coh.dt, T, method="rk4", out=y, support=support[0])

    disc()
    torch.cuda.synchronize(dev)
    support[0] = mask.cpu().numpy() != 0
    for _ in range(warmup):
        disc()
        roll()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        disc()
        roll()
    torch.cuda.synchronize(dev)
    ms_step = (time.perf_counter() - t0) / steps * 1e3

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    n_roof = max(steps, 5)
    gram_ms_t = timed(lambda: MS.gram_ms(coh.x, coh.a, lib, coh.dt, out=(G, B)), n_roof)
    roll_ms_t = timed(roll, n_roof)
    roll_dense_t = timed(lambda: MS.rollout_ms(coh.y0, a_cf, coef, lib, coh.dt, T, method="rk4", out=y), n_roof)
    truth = MS.c3_truth_coef(lib, device=dev)
    rows = N * T
    gflop = 2.0 * (F * (F + 1) / 2 + F * S) * rows          # algorithmic: G upper triangle + B per row
    # issued by gram_ms4_kernel (insite_ms.hip): NB 4x4x4 f64 blocks per row, 16 FMA = 32 flop each -- the C3
    # library's moment cover (csrc/ms4_cover_c3.inc, kMs4CoverNB) or, for other libraries, the column-group form
    # (row group rg <= column group cg over Y = Theta, Z = [Theta | xdot])
    rg, cg = (F + 3) // 4, (F + S + 3) // 4
    nb4 = rg * cg - rg * (rg - 1) // 2
    if (F, S) == (22, 5):
        import re
        inc = open(os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd",
                                "csrc", "ms4_cover_c3.inc")).read()
        nb4 = int(re.search(r"kMs4CoverNB = (\d+)", inc).group(1))
    mfma_flop = nb4 * 32.0 * rows
    roll_bytes = T * N * S * 4 + N * S * 4 + T * ((N + 31) // 32) * 4
    gram_bytes = T * N * S * 4 + T * ((N + 31) // 32) * 4
    out = {
        "metric": METRIC, "value": N / (ms_step * 1e-3), "unit": "patient-trajectories/s", "n_gpus": 1,
        "steps": steps, "warmup": warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32 (storage, rollout) / f64 (Gram, STLSQ)",
        "data": "synthetic: on-device C3 cohort (planted 5-state system, Markov treatment, RK4-10 truth)",
        "config": {"workload": f"C3: 5-state + binary treatment, {N // 1000}k patients x {T} steps: discovery "
                               f"(S-state Gram on f64 MFMA + STLSQ per state) + RK4 counterfactual rollout",
                   "patients": N, "T": T, "states": S, "library_terms": F,
                   "support_equals_truth": bool(torch.equal(mask != 0, truth != 0))},
        "roofline": {"kernel": "gram_ms4_kernel", "bound": "mfma", "achieved": gflop / (gram_ms_t * 1e-3) / 1e12,
                     "peak": 78.6, "unit": "TFLOP/s", "frac": gflop / (gram_ms_t * 1e-3) / 1e12 / 78.6,
                     "traffic": traffic_for("c3", "gram_ms4_kernel", args=args), "avg_launch_ms": gram_ms_t,
                     "issued_mfma_TFLOPs": mfma_flop / (gram_ms_t * 1e-3) / 1e12, "mfma_blocks_per_row": nb4,
                     "hbm_GBps": gram_bytes / (gram_ms_t * 1e-3) / 1e9},
        "rollout": {"kernel": "ms_rollout_sparse (hipRTC, support-specialised; rk4, fp32)", "bound": "hbm",
                    "avg_launch_ms": roll_ms_t, "model_terms": int(support[0].sum()),
                    "algorithmic_bytes": roll_bytes, "achieved_GBps": roll_bytes / (roll_ms_t * 1e-3) / 1e9,
                    "frac": roll_bytes / (roll_ms_t * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                    "dense_kernel_avg_launch_ms": roll_dense_t},
    }
    if parity:
        out["parity"] = c3_parity(coh, a_cf, lib, T, G, B, coef, mask, y)
    return out


C5_COEF = (-1.1108, -0.1454, -1.0235)   # the EQ_4_C model of the reference log (final_with_insite.txt:182)
# fp64 VALU work of one RK45 step attempt (rollout_rk45_kernel, rk45_ref.rk45_interval): 6 stage RHS
# evaluations of alpha + beta*y (1 FMA each), 21 stage-combination FMAs (Dormand-Prince a_ij), 5th-order
# update (6 FMA), error estimate (7 FMA), error norm (scale, ratio, square: 4 ops), step-size factor
# (rk45_inv_root5: ~20 ops), accept/reject bookkeeping (~6 ops) -> ~71 fp64 ops, 2 flops per FMA:
RK45_FLOP_PER_ATTEMPT = 2 * (6 + 21 + 6 + 7) + 4 + 20 + 6
FP64_VALU_PEAK_TFLOPS = 78.6            # MI355X spec FP64 vector


def _cpu_rk45_chunk(bounds):
    from oracle import rk45_ref as K
    lo, hi = bounds
    d = _CPU
    K.rollout_rk45(d["y0"][lo:hi], d["u"][lo:hi], d["arm"][lo:hi], d["t"][lo:hi], d["n"][lo:hi], d["coef"], d["exps"])
    return hi - lo


def _cpu_rk45_ivp_chunk(bounds):
    """scipy.integrate.solve_ivp(RK45, rtol = atol = 1.4e-8) over every observation interval of each patient
    with the interval's arm held (the call the restatement in oracle/rk45_ref.py is pinned to)."""
    from scipy.integrate import solve_ivp
    from oracle import rk45_ref as K
    lo, hi = bounds
    d = _CPU
    acc = 0.0
    for p in range(lo, hi):
        al, be = K.patient_rates(d["u"][p], d["coef"], d["exps"])
        y = float(d["y0"][p])
        for k in range(int(d["n"][p]) - 1):
            a = int(d["arm"][p, k])
            t0, t1 = float(d["t"][p, k]), float(d["t"][p, k + 1])
            if t1 > t0:
                sol = solve_ivp(lambda t, v, a=a: al[a] + be[a] * v, (t0, t1), [y], method="RK45",
                                rtol=K.RTOL, atol=K.ATOL)
                y = float(sol.y[0, -1])
        acc += y
    return acc


def c5_cpu_baseline(n_sample, seed, ivp_per_worker=40):
    """oracle/rk45_ref.py (scipy 1.15 RK45 restated, pinned to solve_ivp at 1e-13) on a process pool over
    a bounded sample of the C5 workload, before any GPU context exists."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    from oracle import rk45_ref as K
    info = host_info()
    W = info["workers"]
    rng = np.random.default_rng(seed)
    t, n = K.irregular_grid(n_sample, rng)
    coef = np.zeros((2, 7))
    coef[0, 4], coef[1, 1], coef[1, 5] = C5_COEF
    _CPU.update(t=t, n=n, y0=rng.uniform(1, 50, n_sample), u=rng.normal(0.5, 0.05, (n_sample, 2)),
                arm=rng.integers(0, 2, (n_sample, t.shape[1])), coef=coef, exps=R.poly_library(3, 2, True))
    chunks = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(n_sample), W) if c.size]
    n_ivp = min(n_sample, ivp_per_worker * W)
    ivp_chunks = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(n_ivp), W) if c.size]
    with worker_pool(mp.get_context("fork"), W, _cpu_worker_init) as pool:
        pool.map(abs, range(W))
        t0 = time.perf_counter()
        pool.map(_cpu_rk45_chunk, chunks)
        el = time.perf_counter() - t0
        t1 = time.perf_counter()
        pool.map(_cpu_rk45_ivp_chunk, ivp_chunks)
        el_ivp = time.perf_counter() - t1
    return {"value": n_sample / el, "unit": "patient-trajectories/s", "cores": W, "kind": "port",
            "sample": f"oracle/rk45_ref.py (scipy RK45 restated) on {n_sample} irregular-grid patients over {W} "
                      f"worker processes, {el:.2f} s", "host": info,
            "scipy_solve_ivp": {
                "value": n_ivp / el_ivp, "unit": "patient-trajectories/s", "cores": W,
                "kind": "scipy.integrate.solve_ivp(method='RK45', rtol=atol=1.4e-8) per observation interval",
                "sample": f"{n_ivp} irregular-grid patients on {W} workers in {el_ivp:.2f} s (one solve_ivp call per "
                          f"interval, arm held over it, as the reference integrates per interval); the rate "
                          f"extrapolates linearly in patients"}}


def _binned_divergence(st, chunk):
    """Wave divergence (sum of per-wave max / sum of attempts) if the lanes took the rows sorted by attempt count inside
    consecutive ``chunk``-row ranges (descending), whole waves of 64."""
    n = st.numel() // chunk * chunk
    srt = torch.sort(st[:n].view(-1, chunk), dim=1, descending=True).values.reshape(-1)
    w = srt[: n // 64 * 64].view(-1, 64)
    return float((w.max(dim=1).values.mean() / w.mean()).item()) if w.numel() else None


def c5_main(args):
    """Configuration C5 (BASELINE.json configs[4]): PK/PD EQ_4_C model rolled out with the adaptive
    RK45 controller (scipy solve_ivp semantics, rtol = atol = 1.4e-8) on per-patient irregular grids
    (20..60 observations on [0, 10]), 1M patients sharded over the ranks (strong scaling: configs[4] fixes
    1M patients on 8 GPUs; no collective on the data path); arms switch per interval.  One step = one
    rollout of every patient.  Lane-level step-size control: waves run until their slowest lane finishes."""
    cpu = None
    if os.environ.get("WORLD_SIZE", "1") == "1" and not args.no_cpu_baseline:
        cpu = c5_cpu_baseline(min(10 * args.cpu_sample, 100_000), args.seed + 4)   # ~10 s on 16 workers
    world, rank, dev = dist_setup()
    from insite_amd import ops, cohort
    from insite_amd import dist as idist
    from insite_amd.library import polynomial_library
    N_total = args.patients if args.patients != 100_000 else 1_000_000
    lo, hi = idist.shard_bounds(N_total, rank, world)
    N = hi - lo
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed * 1000 + 5 + rank)
    t_obs, n_obs = cohort.irregular_grid(N, seed=args.seed * 1000 + 4 + rank, device=dev)
    Tm = t_obs.size(0)
    # patient-major grids, arms and outputs (INSITE_LAYOUT_PATIENT_MAJOR_BITS)
    t_dev = torch.nan_to_num(t_obs, nan=0.0).t().contiguous()
    u = torch.randn((N, 2), generator=g, device=dev, dtype=torch.float64) * 0.05 + 0.5
    y0 = torch.rand((N,), generator=g, device=dev, dtype=torch.float64) * 49 + 1
    arm = (torch.rand((N, Tm), generator=g, device=dev) < 0.5).to(torch.int8)
    bits = ops.pack_arm_bits(arm, Tm)
    lib = polynomial_library(2, 2, True)
    coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
    coef[0, 4], coef[1, 1], coef[1, 5] = C5_COEF
    # rows padded to whole 64-B sectors (ld 64): the kernel stages each lane's outputs per sector
    y = torch.empty((N, (Tm + 7) // 8 * 8), dtype=torch.float64, device=dev)[:, :Tm]
    steps = torch.zeros((N,), dtype=torch.int32, device=dev)

    order = not args.rk45_identity_order
    by_attempts = order and args.rk45_bin == "attempts"

    # binning (the counting sort, by n_obs or by the previous step's attempt counts) runs inside every step; the plan
    # packs the two C calls once
    plan = ops.plan_rollout_rk45(y0, u, bits, t_dev, n_obs, coef, lib, out=y, steps=steps, layout="patient",
                                 order="attempts" if by_attempts else order)
    lane_order = ((lambda: ops.rk45_order(steps, ops.RK45_ATTEMPT_BINS - 1)) if by_attempts
                  else (lambda: ops.rk45_order(n_obs, Tm)))

    def run():
        plan()

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ms_step = idist.max_over_ranks(time.perf_counter() - t0, dev) / args.steps * 1e3
    # per-launch duration with HIP events on the launch stream (instrumented pass after the timed region)
    st_ = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(max(args.steps, 5))]
    for e0, e1 in evs:
        e0.record(st_)
        run()
        e1.record(st_)
    torch.cuda.synchronize(dev)
    launch_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    st = steps.to(torch.float64)
    # waves as the kernel formed them: lanes take rows in the binned order (ops.rk45_order)
    per_wave = (st[lane_order().long()] if order else st)[: N // 64 * 64].view(-1, 64)
    intervals = (n_obs - 1).to(torch.float64)
    attempts = float(st.sum())
    flop = attempts * RK45_FLOP_PER_ATTEMPT
    issued = float(per_wave.max(dim=1).values.sum()) * 64 * RK45_FLOP_PER_ATTEMPT   # lanes idle behind the slowest
    out = {
        "metric": METRIC, "value": N_total / (ms_step * 1e-3), "unit": "patient-trajectories/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: irregular grids T_p ~ U{20..60} on [0,10], EQ_4_C statics, random per-interval arms",
        "config": {"workload": f"C5: adaptive RK45 (rtol=atol=1.4e-8) on irregular grids, {N_total // 1000}k patients",
                   "patients_total": N_total, "patients_per_gpu": N, "max_obs": Tm,
                   "mean_intervals": float(intervals.mean()), "parallelism": f"patient-shard x{world}"},
        "roofline": {"kernel": "rollout_rk45_kernel", "bound": "valu-f64", "unit": "TFLOP/s",
                     "achieved": flop / (launch_ms * 1e-3) / 1e12, "peak": FP64_VALU_PEAK_TFLOPS,
                     "frac": flop / (launch_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS,
                     "traffic": c5_traffic_calibrated(args),
                     "traffic_method": "PMC FETCH_SIZE / WRITE_SIZE of the kernel (profiles/traffic_r05.json, else r04) "
                                       "divided by this access shape's calibration factors (profiles/r05/c5cal/"
                                       "calibration.json: window-refill reads 0.617, 64-B sector writes 1.081), not "
                                       "the wide-streaming x2",
                     "traffic_blanket_x2": traffic_for("c5", "rollout_rk45_flat_kernel", args=args),
                     "data_bytes": float(N * (8 * 3 + 4) + n_obs.to(torch.float64).sum().item() * 8 * 2
                                         + N * ((Tm + 30) // 32) * 4),
                     "avg_launch_ms": launch_ms, "flop_per_attempt": RK45_FLOP_PER_ATTEMPT,
                     "issued_incl_divergence_TFLOPs": issued / (launch_ms * 1e-3) / 1e12,
                     "algorithmic_bytes": N * (8 * 3 + 4) + N * Tm * 8 * 2 + N * ((Tm + 30) // 32) * 4,
                     "achieved_GBps": (N * (8 * 3 + 4) + N * Tm * 8 * 2 + N * ((Tm + 30) // 32) * 4) / (launch_ms * 1e-3) / 1e9},
        "rk45": {"mean_attempts_per_patient": float(st.mean()),
                 "mean_attempts_per_interval": float(st.sum() / intervals.sum()),
                 "wave_divergence": float((per_wave.max(dim=1).values.mean() / per_wave.mean()).item()),
                 #  the same figure under its explicit name: a wave's flat loop runs its slowest
                 # lane's attempt count, so sum over waves of max / sum of attempts is the issued-work inflation
                 "attempts_max_over_mean_per_wave": float((per_wave.max(dim=1).values.mean() / per_wave.mean()).item()),
                 "lane_binning": ("by the previous step's per-patient attempt counts (a C5 step re-rolls the same "
                                  "cohort; the first call bins zeros)") if by_attempts else
                                 ("by n_obs" if order else "identity"),
                 # with n_obs binning: what attempt binning inside the same 4096-row chunks would give
                 "attempts_max_over_mean_if_binned_by_attempts": _binned_divergence(st, 4096),
                 "rhs_evals_per_s": float(st.sum() * 6 / (launch_ms * 1e-3))},
    }
    if world == 1 and not args.no_parity:
        out["parity"] = c5_parity(y0, u, arm, t_obs, n_obs, coef, lib, y, steps,
                                  lane_order() if order else torch.arange(N, device=dev))
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        emit(out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# --------------------------------------------------------------------------------------------------
# Oracle parity of the timed cohorts (the metric's "RMSE vs CPU ref" for every line): after
# the timed region, a sample of the rows the last timed step computed goes through the oracle restatement on a
# SPAWNED pool of the host's workers (fresh interpreters that never touch the GPU; fork is not safe once this
# process holds a GPU context).  The checker only -- nothing here is timed or feeds the product path.
# --------------------------------------------------------------------------------------------------
def _par_init():
    _cpu_worker_init()
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)


def parity_map(fn, jobs):
    import multiprocessing as mp
    W = min(host_info()["workers"], len(jobs))
    if W <= 1:
        _par_init()
        return [fn(j) for j in jobs]
    with worker_pool(mp.get_context("spawn"), W, _par_init) as pool:
        return pool.map(fn, jobs)


def sample_rows(N, n, seed, extra=()):
    """A fixed sample of row indices: n random rows, the first and last 64 and any ``extra`` (e.g. the first and
    last lanes of a binned order)."""
    rng = np.random.default_rng(seed)
    idx = [rng.choice(N, min(n, N), replace=False), np.arange(min(64, N)), np.arange(max(0, N - 64), N)]
    idx += [np.asarray(e, dtype=np.int64).reshape(-1) for e in extra]
    return np.unique(np.concatenate(idx))


def _par_refine_job(job):
    from oracle import insite_refine_ref as Q
    V, arm, u, sl, c0, ex, dt, lam, tau, n_in = job[:10]
    rev = bool(job[10]) if len(job) > 10 else False
    out = [Q.refine_patient(V[i], arm[i], u[i], int(sl[i]), c0, ex, dt, lam, tau, n_inputs=n_in,
                            revert_on_zoom_fail=rev) for i in range(V.shape[0])]
    return (np.stack([o[0] for o in out]), np.stack([np.asarray(o[1]).reshape(-1) for o in out]),
            np.array([o[2] for o in out]), np.array([o[3] for o in out]))


def insite_parity(V, arm, u, sl, c0, lib, dt, lam, tau, preds, coef, status, iters, n_sample=4096, seed=13,
                  extra=(), revert=False):
    """The INSITE lines' parity: ``n_sample`` rows of the timed cohort (plus ``extra``, e.g. the first / last lanes
    of the binned order) through oracle/insite_refine_ref.refine_patient (the reference's jax BFGS restated,
    sindy.py:587-665, 781-794) against the rows the last timed step wrote: per-row status and iteration count
    equality (reported as fractions: the GPU's closed-form objective scans round differently from the sub-step
    form, so an ill-conditioned row can take another BFGS path), refined coefficients, predictions."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    N, T = V.shape
    idx = sample_rows(N, n_sample, seed, extra)
    it = torch.as_tensor(idx, device=V.device)

    def h(t):
        return t.index_select(0, it).cpu().numpy()
    Vh, ah, uh, slh = h(V), h(arm).astype(np.int64), h(u), h(sl)
    ex = lib.exps.astype(np.int64)
    W = host_info()["workers"]
    parts = [c for c in np.array_split(np.arange(idx.size), 4 * W) if c.size]
    t0 = time.perf_counter()
    res = parity_map(_par_refine_job, [(Vh[c], ah[c], uh[c], slh[c], np.asarray(c0, dtype=np.float64), ex, dt, lam,
                                        tau, int(lib.n_inputs), revert) for c in parts])
    el = time.perf_counter() - t0
    P, C = np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])
    S, I = np.concatenate([r[2] for r in res]), np.concatenate([r[3] for r in res])
    gp, gc, gs, gi = h(preds), h(coef).reshape(idx.size, -1), h(status), h(iters)
    same = gs == S
    ref_ = S >= 0
    d = gp - P
    rel = np.abs(d) / np.maximum(np.abs(P), 1e-300)
    return {"oracle": "oracle/insite_refine_ref.refine_patient (jax BFGS + line search + zoom restated, numpy; "
                      "sindy.py:587-665, 781-794)",
            "cohort": f"the last timed step's rows ({N} x {T})", "rows_sampled": int(idx.size),
            "refined_rows": int(ref_.sum()), "status_equal_frac": float(same.mean()),
            "iterations_equal_frac": float((gi[ref_] == I[ref_]).mean()) if ref_.any() else 1.0,
            "pred_rmse": float(np.sqrt(np.mean(d ** 2))), "pred_max_rel": float(rel.max()),
            "pred_max_rel_status_equal": float(rel[same].max()) if same.any() else None,
            "status_mismatch_pairs_gpu_oracle": {f"{a}/{b}": int(((gs == a) & (S == b)).sum())
                                                 for a, b in sorted(set(zip(gs[~same].tolist(), S[~same].tolist())))},
            "coef_linf": float(np.abs(gc - C).max()),
            "coef_linf_status_equal": float(np.abs(gc - C)[same].max()) if same.any() else None,
            "oracle_seconds": el,
            **({"revert_on_zoom_fail": True,
                # the status-mismatch rows under the literal revert (sindy.py:628-631): one side keeps c0, the other
                # its BFGS iterate, so their predictions differ by the refinement itself -- reported, not toleranced
                "mismatch_rows": int((~same).sum()),
                "pred_rmse_status_equal": float(np.sqrt(np.mean(d[same] ** 2))) if same.any() else None,
                "pred_max_rel_status_mismatch": float(rel[~same].max()) if (~same).any() else None,
                "mismatch_reverted_side_is_c0": bool(all(
                    np.array_equal((gc if gs[i] == 3 else C)[i], np.asarray(c0, dtype=np.float64).reshape(-1)[:gc.shape[1]])
                    for i in np.flatnonzero(~same) if 3 in (gs[i], S[i])))} if revert else {}),
            "tolerances": {"status_equal_frac": 0.995, "pred_rmse": 1e-6, "coef_linf": 1e-7}}


def _par_rk45_job(job):
    from oracle import rk45_ref as K
    return K.rollout_rk45(*job)


def c5_parity(y0, u, arm, t_obs, n_obs, coef, lib, y, steps, order, n_sample=4096, seed=5):
    """C5: sampled rows of the timed cohort (first / last lanes of the binned order included) through
    oracle/rk45_ref.rollout_rk45 (scipy 1.15 solve_ivp RK45 restated, pinned to solve_ivp at 1e-13) against the
    trajectories and per-patient attempt counts the last timed launch wrote."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    N = y0.numel()
    o = order.cpu().numpy()
    idx = sample_rows(N, n_sample, seed, extra=(o[:64], o[-64:], o[N // 2 - 32:N // 2 + 32]))
    it = torch.as_tensor(idx, device=y0.device)
    tn = t_obs.index_select(1, it).t().contiguous().cpu().numpy()
    nn, y0h, uh, ah = (v.index_select(0, it).cpu().numpy() for v in (n_obs, y0, u, arm))
    ch, ex = coef.cpu().numpy(), lib.exps.astype(np.int64)
    parts = [c for c in np.array_split(np.arange(idx.size), 4 * host_info()["workers"]) if c.size]
    t0 = time.perf_counter()
    res = parity_map(_par_rk45_job, [(y0h[c], uh[c], ah[c], tn[c], nn[c], ch, ex) for c in parts])
    el = time.perf_counter() - t0
    ref = np.concatenate([r[0] for r in res])
    rs = np.concatenate([r[1] for r in res])
    got = y.index_select(0, it).cpu().numpy()[:, :ref.shape[1]]
    st = steps.index_select(0, it).cpu().numpy()
    valid = ~np.isnan(ref)
    same = st == rs
    d = np.where(valid, got - ref, 0.0)
    rel = np.abs(d) / np.where(valid, np.abs(ref), 1.0)
    return {"oracle": "oracle/rk45_ref.rollout_rk45 (scipy 1.15 RK45 restated, pinned to solve_ivp)",
            "cohort": f"the last timed launch's rows ({N} patients)", "rows_sampled": int(idx.size),
            "attempts_equal_frac": float(same.mean()), "y_rmse": float(np.sqrt(np.sum(d ** 2) / valid.sum())),
            "y_max_rel": float(rel.max()), "y_max_rel_attempts_equal": float(rel[same].max()) if same.any() else None,
            "oracle_seconds": el, "tolerances": {"y_rmse": 1e-6, "y_max_rel": 1e-9, "attempts_equal_frac": 0.999}}


def _unpack_bits_rows(bits, idx, T):
    """bit words -> [n, T] int64 arms of the rows idx (tensor on its device): time-major [T, W] int32, or tile-major
    [ceil(N/64), S >= T, 2] int32 (ops.tile_major_bits)."""
    if bits.dim() == 3:
        words = bits[idx // 64, :T, (idx // 32) % 2].t()                        # [T, n]
    else:
        words = bits[:T].index_select(1, idx // 32)
    return ((words >> (idx % 32).to(torch.int32)[None, :]) & 1).t().contiguous().cpu().numpy().astype(np.int64)


def _par_gram_job(job):
    from oracle import insite_ref as R
    return R.gram_moments_vectorized(*job)


def _par_ppfit_roll_job(job):
    from oracle import insite_ref as R
    x, u, arm, rows, dt, ex, gc, y0, arms_cf = job
    pc, pm, pi = R.per_patient_fit(x, u, arm, rows, dt, ex, gc, 0.1, 0.5)
    return pc, pm, pi, R.rollout(y0, u, arms_cf, pc, ex, dt, method="euler5")


def c4_parity(coh, arm_cf, lib, T, gcoef, gmask, pout, y, n_sample=4096, seed=3):
    """C4: the global model against the oracle's Gram-form STLSQ over the WHOLE timed cohort (chunked vectorised
    Gram on the host's workers), and on sampled rows the per-patient refits (oracle/insite_ref.per_patient_fit, the
    LSQIntialMask restatement, pkpd_simulation.py:791-800) and their Euler-5 rollouts (sindy.py:767-778) against
    the refits and the trajectories of the last timed launch."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    N = coh.arm.numel()
    rows = coh.rows.cpu().numpy()
    if not np.all(rows == rows[0]):
        return {"skipped": "ragged rows (the vectorised oracle Gram needs equal rows)"}
    ex = lib.exps.astype(np.int64)
    un, an = coh.u.cpu().numpy(), coh.arm.cpu().numpy().astype(np.int64)
    W = host_info()["workers"]
    bounds = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(N), 2 * W) if c.size]
    t0 = time.perf_counter()
    gb = parity_map(_par_gram_job, [(coh.x[:T, lo:hi].t().contiguous().cpu().numpy(), un[lo:hi], an[lo:hi],
                                     int(rows[0]), coh.dt, ex) for lo, hi in bounds])
    G, b = sum(q[0] for q in gb), sum(q[1] for q in gb)
    cr = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    idx = sample_rows(N, n_sample, seed)
    it = torch.as_tensor(idx, device=coh.x.device)
    xs = coh.x[:T].index_select(1, it).t().contiguous().cpu().numpy()
    us, ars, rws = un[idx], an[idx], rows[idx]
    y0 = coh.y0.index_select(0, it).cpu().numpy()
    acf = _unpack_bits_rows(arm_cf, it, T)
    gc = gcoef.cpu().numpy()
    parts = [c for c in np.array_split(np.arange(idx.size), 4 * W) if c.size]
    res = parity_map(_par_ppfit_roll_job, [(xs[c], us[c], ars[c], rws[c], coh.dt, ex, gc, y0[c], acf[c])
                                           for c in parts])
    el = time.perf_counter() - t0
    pc = np.concatenate([r[0] for r in res])
    pm = np.concatenate([r[1] for r in res])
    pi = np.concatenate([r[2] for r in res])
    yr = np.concatenate([r[3] for r in res])
    got_y = y.index_select(1, it).t().cpu().numpy()
    d = got_y - yr
    gpc = pout[0].index_select(0, it).cpu().numpy()
    return {"oracle": "oracle/insite_ref.py (gram_moments_vectorized + stlsq_gram over the whole cohort; "
                      "per_patient_fit + rollout euler5 on the sample)",
            "cohort": f"the timed cohort ({N} x {T})", "rows_sampled": int(idx.size),
            "global_support_equal": bool(np.array_equal(gmask.cpu().numpy() != 0, cr != 0)),
            "global_coef_linf": float(np.abs(gc - cr).max()),
            "per_patient_support_equal_frac": float((pout[1].index_select(0, it).cpu().numpy() == pm).all(1).mean()),
            "per_patient_iterations_equal_frac": float((pout[2].index_select(0, it).cpu().numpy() == pi).mean()),
            "per_patient_coef_linf": float(np.abs(gpc - pc).max()),
            "y_rmse": float(np.sqrt(np.mean(d ** 2))),
            "y_max_rel": float((np.abs(d) / np.maximum(np.abs(yr), 1e-300)).max()), "oracle_seconds": el,
            "tolerances": {"global_coef_linf": 1e-8, "per_patient_coef_linf": 1e-8, "y_rmse": 1e-6}}


def _par_seg_gram_job(job):
    from oracle import segments_ref as S
    return S.gram_segments_vectorized(*job)


def _par_roll_job(job):
    from oracle import insite_ref as R
    y0, u, arms, coef, ex, dt, method = job
    return R.rollout(y0, u, arms, coef, ex, dt, method=method)


def f4_parity(coh, arm_cf, lib, T, coef, mask, y, n_sample=4096, seed=31):
    """F4: the four per-arm models against the oracle's segment Gram (oracle/segments_ref.gram_segments_vectorized,
    the reference's segment walk in index form, pkpd/utils.py:433-462, 607-637) over the WHOLE timed cohort + STLSQ
    (threshold 0.001), and the Euler-5 4-arm rollout of sampled rows against the trajectories of the last step."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    N = coh.u.size(0)
    ex = lib.exps.astype(np.int64)
    un = coh.u.cpu().numpy()
    sl = coh.seq_len.cpu().numpy().astype(np.int64)
    W = host_info()["workers"]
    bounds = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(N), 2 * W) if c.size]
    t0 = time.perf_counter()
    gb = parity_map(_par_seg_gram_job, [(coh.x[:, lo:hi].t().contiguous().cpu().numpy(), un[lo:hi],
                                         coh.arm[:, lo:hi].t().contiguous().cpu().numpy().astype(np.int64), sl[lo:hi],
                                         coh.dt, ex) for lo, hi in bounds])
    G, b = sum(q[0] for q in gb), sum(q[1] for q in gb)
    cr = np.stack([R.stlsq_gram(G[k], b[k], 0.001, 0.5)[0] for k in range(4)])
    idx = sample_rows(N, n_sample, seed)
    it = torch.as_tensor(idx, device=coh.x.device)
    y0 = coh.x[0].index_select(0, it).cpu().numpy()
    acf = arm_cf[:T].index_select(1, it).t().contiguous().cpu().numpy().astype(np.int64)
    parts = [c for c in np.array_split(np.arange(idx.size), 4 * W) if c.size]
    yr = np.concatenate(parity_map(_par_roll_job, [(y0[c], un[idx][c], acf[c], cr, ex, coh.dt, "euler5")
                                                   for c in parts]))
    el = time.perf_counter() - t0
    d = y.index_select(1, it).t().cpu().numpy() - yr
    return {"oracle": "oracle/segments_ref.gram_segments_vectorized + insite_ref.stlsq_gram over the whole cohort; "
                      "insite_ref.rollout euler5 on the sample",
            "cohort": f"the timed cohort ({N} x {T}, 4 arms)", "rows_sampled": int(idx.size),
            "support_equal": bool(np.array_equal(mask.cpu().numpy() != 0, cr != 0)),
            "coef_linf": float(np.abs(coef.cpu().numpy() - cr).max()),
            "y_rmse": float(np.sqrt(np.mean(d ** 2))),
            "y_max_rel": float((np.abs(d) / np.maximum(np.abs(yr), 1e-300)).max()), "oracle_seconds": el,
            "tolerances": {"coef_linf": 1e-8, "y_rmse": 1e-6}}


def _par_ms_roll_job(job):
    from oracle import multistate_ref as M
    y0, a, coef, ex, dt = job
    return M.ms_rollout(y0, a, coef, ex, dt, "rk4")


def c3_parity(coh, a_cf, lib, T, G, B, coef, mask, y, n_sample=2048, seed=23):
    """C3: the Gram of sampled sub-cohorts (first tile, an unaligned middle range, the partial last tile) through
    the product kernel against oracle/multistate_ref.ms_gram, the STLSQ of the timed step's full Gram against
    ms_stlsq, and the fp32 RK4 rollout of sampled rows against ms_rollout (fp64)."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from insite_amd import multistate as MS
    from insite_amd import ops
    from oracle import multistate_ref as M
    N = coh.x.size(2)
    ex = lib.exps.astype(np.int64)

    def unpack(bits, lo, hi):
        b_ = bits[:T].cpu().numpy().view(np.uint32)
        r = np.arange(lo, hi)
        return ((b_[:, r >> 5] >> (r & 31).astype(np.uint32)) & 1).T.astype(np.int8)
    t0 = time.perf_counter()
    cuts = [(0, 64), (N // 2 - 32, N // 2 + 64), (max(0, N - 96), N)]
    gmax = 0.0
    for lo, hi in cuts:
        lo -= lo % 32
        g_, b_ = MS.gram_ms(coh.x[:, :, lo:hi].contiguous(), coh.a[:, lo // 32:(hi + 31) // 32].contiguous(), lib,
                            coh.dt, workspace=ops.Workspace())
        xn = np.transpose(coh.x[:, :, lo:hi].cpu().numpy(), (2, 0, 1))
        Gr, Br = M.ms_gram(xn, unpack(coh.a, lo, hi), np.full(hi - lo, T), coh.dt, ex)
        gmax = max(gmax, float(np.max(np.abs(g_.cpu().numpy() - Gr) / np.maximum(np.abs(Gr), 1.0))),
                   float(np.max(np.abs(b_.cpu().numpy() - Br) / np.maximum(np.abs(Br), 1.0))))
    c_ref, m_ref, _ = M.ms_stlsq(G.cpu().numpy(), B.cpu().numpy())
    idx = sample_rows(N, n_sample, seed)
    it = torch.as_tensor(idx, device=coh.x.device)
    y0 = coh.y0.index_select(1, it).t().cpu().numpy().astype(np.float64)
    words = a_cf[:T].index_select(1, it // 32)
    acf = ((words >> (it % 32).to(torch.int32)[None, :]) & 1).t().contiguous().cpu().numpy().astype(np.int8)
    cg = coef.cpu().numpy()
    parts = [c for c in np.array_split(np.arange(idx.size), 4 * host_info()["workers"]) if c.size]
    yr = np.concatenate(parity_map(_par_ms_roll_job, [(y0[c], acf[c], cg, ex, coh.dt) for c in parts]))
    el = time.perf_counter() - t0
    got = np.transpose(y.index_select(2, it).cpu().numpy(), (2, 0, 1)).astype(np.float64)
    rel = np.abs(got - yr) / np.maximum(np.abs(yr), 1e-2)
    return {"oracle": "oracle/multistate_ref.py (ms_gram on sampled sub-cohorts, ms_stlsq on the step's Gram, "
                      "ms_rollout rk4 fp64 on sampled rows)",
            "cohort": f"the timed cohort ({N} x {T} x {lib.n_states})", "rows_sampled": int(idx.size),
            "gram_max_rel_sampled_tiles": gmax, "support_equal": bool(np.array_equal(mask.cpu().numpy() != 0, m_ref)),
            "coef_linf": float(np.abs(cg - c_ref).max()),
            "y_max_rel_fp32_vs_fp64": float(rel.max()), "y_rmse": float(np.sqrt(np.mean((got - yr) ** 2))),
            "oracle_seconds": el,
            "tolerances": {"gram_max_rel_sampled_tiles": 1e-10, "coef_linf": 1e-8, "y_max_rel_fp32_vs_fp64": 1e-4}}


def _cpu_pp_init(*data):
    _cpu_worker_init()
    _CPU["pp"] = data


def _cpu_pp_fit_chunk(bounds):
    sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    lo, hi = bounds
    xs, us, ar, rw, dt, ex, gc = _CPU["pp"]
    R.per_patient_fit(xs[lo:hi], us[lo:hi], ar[lo:hi], rw[lo:hi], dt, ex, gc, 0.1, 0.5)
    return hi - lo


def _cpu_refine_chunk(bounds):
    from oracle import insite_ref as R
    from oracle import insite_refine_ref as Q
    lo, hi = bounds
    d = _CPU
    ex = R.poly_library(3, 2, True)
    for i in range(lo, hi):
        Q.refine_patient(d["V"][i], d["arm"][i], d["u"][i], int(d["sl"][i]), d["c0"], ex, d["dt"], 10.0, 5)
    return hi - lo


def insite_cpu_baseline(seed, per_worker=2000):
    """Bounded CPU sample of the F2 workload on the host's workers: the oracle's restatement of the jax
    BFGS refinement (oracle/insite_refine_ref.py) on rows of the same shape (EQ_4_C, T = 60, seq_len
    U{1..59}, arm flipped at a random step), per_worker rows per worker."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    info = host_info()
    W = info["workers"]
    n = W * per_worker
    rng = np.random.default_rng(seed + 9)
    T = 60
    p = R.draw_params(n, "EQ_4_C", rng)
    sim = R.simulate_factual(p, T, rng, "EQ_4_C", 2.0)
    arm0 = sim["treatment_application"][:, 0].astype(np.int64)
    flip = rng.integers(1, T, size=(n, 1))
    c0 = np.zeros((2, 7))
    c0[0, 4], c0[1, 1], c0[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    _CPU.update(V=sim["cancer_volume"][:, :T], arm=np.where(np.arange(T)[None, :] >= flip, 1 - arm0[:, None],
                                                             arm0[:, None]).astype(np.int8),
                u=np.stack([sim["observed_static_c_0"], sim["observed_static_c_1"]], axis=1),
                sl=rng.integers(1, T, size=n), c0=c0, dt=10.0 / T)
    chunks = [(int(a[0]), int(a[-1]) + 1) for a in np.array_split(np.arange(n), W) if a.size]
    with worker_pool(mp.get_context("fork"), W, _cpu_worker_init) as pool:
        pool.map(abs, range(W))
        t0 = time.perf_counter()
        pool.map(_cpu_refine_chunk, chunks)
        el = time.perf_counter() - t0
    return {"value": n / el, "unit": "patient-trajectories/s", "cores": W, "kind": "port",
            "sample": f"oracle/insite_refine_ref.py (jax BFGS restated, numpy) on {n} EQ_4_C rows (T = 60, seq_len "
                      f"U{{1..59}}) over a {W}-process pool, {el:.2f} s", "host": info}


def insite_rows(N, T, seed, dev):
    """The INSITE line's rows (also tests/test_gpu_insite.py's bench-size parity cohort): an on-device EQ_4_C
    cohort, patient-major V [N, T], per-step int8 arms (the factual arm flipped at a random step), seq_len
    U{1..T-1}, and the global model of the EQ_4_C log (final_with_insite.txt:182).  Returns
    (cohort, V, arm, seq_len, c0, dt)."""
    from insite_amd import cohort
    coh = cohort.synthetic_pkpd(N, T, seed=seed + 9, device=dev, equation="EQ_4_C")
    V = coh.x[:, :T].contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 10)
    flip = torch.randint(1, T, (N, 1), generator=g, device=dev)
    arm = torch.where(torch.arange(T, device=dev)[None, :] >= flip, 1 - coh.arm[:, None].to(torch.int64),
                      coh.arm[:, None].to(torch.int64)).to(torch.int8).contiguous()
    sl = torch.randint(1, T, (N,), generator=g, device=dev, dtype=torch.int32)
    c0 = np.zeros((2, coh.lib.n_terms))
    c0[0, 4], c0[1, 1], c0[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243  # log :182
    return coh, V, arm, sl, c0, 10.0 / T


def insite_main(args):
    """INSITE per-patient refinement (reference sindy.py:433-715): every row of a
    counterfactual evaluation set refines the global EQ_4_C model by BFGS on its observed prefix
    (tau = 5) and rolls its model out with Euler-5.  Rows: PK/PD trajectories of T = 60 observations,
    sequence lengths U{1..59}, per-step arms (factual arm, flipped at a random step).  One step = one
    refinement of every row (1M rows; the reference's tau-step test set has 59,000)."""
    # the CPU leg first, while this process has no GPU context (its worker pool forks)
    cpu = None if args.no_cpu_baseline else insite_cpu_baseline(args.seed)
    from insite_amd import ops
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = args.patients if args.patients != 100_000 else 1_000_000
    T = 60
    coh, V, arm, sl, c0, dt = insite_rows(N, T, args.seed, dev)

    # the product's binned path as a prepared plan: the seq_len sort and the refinement on the patient-major rows
    # (insite_refine_rows_f64, ABI 9: 2 C calls, no host synchronisation) inside every step
    # --insite-order nfev (default): the lanes binned by window AND by the evaluation counts of the previous step
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, order=args.insite_order)
    plan_prep = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, rows=False)   # ABI 8 route

    def run(mode):   # "binned": rows binned by seq_len on the device (inside every step)
        if mode == "binned":
            return plan()
        if mode == "prepare":
            return plan_prep()
        return ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, binned=False)

    def timed(mode):
        for _ in range(args.warmup):
            run(mode)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            r = run(mode)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / args.steps * 1e3, r

    only = args.insite_only_binned            # (profiling: the other routes' launches stay out of the counters)
    ms_identity, _ = (None, None) if only else timed("identity")
    ms_prepare, prep_out = (None, None) if only else timed("prepare")
    ms_step, (preds, coef, status, iters) = timed("binned")    # the product default: rows binned by seq_len
    eager = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, binned=True)
    plan_eq = all(bool(torch.equal(a, b)) for a, b in zip(eager, (preds, coef, status, iters)))
    prep_eq = None if only else all(bool(torch.equal(a, b)) for a, b in zip(prep_out, (preds, coef, status, iters)))
    st = status.cpu().numpy()
    it = iters.cpu().numpy()
    # roofline: the refinement kernel alone (the plan's second call, its lane order computed by the steps above),
    # HIP events on its stream; its work = every objective/gradient evaluation (nfev per row, counted by the kernel
    # on one untimed launch) x the row's K-step window x flops per sensitivity step
    kst = torch.cuda.current_stream(dev)
    # the kernel's call index in the plan: [sort, rows kernel] in rows mode, [sort, prepare, kernel, finish] when the
    # row kernel refused the shape (prepare mode)
    kidx_ins = plan.kernel_call

    def kern():
        plan.call(kidx_ins, kst)

    for _ in range(2):
        kern()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(kst)
    for _ in range(args.steps):
        kern()
    e1.record(kst)
    torch.cuda.synchronize(dev)
    kern_ms = e0.elapsed_time(e1) / args.steps
    nf_row = torch.empty((N,), dtype=torch.int32, device=dev)
    plan_nf = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, nfev=nf_row)
    p2, _, s2, i2 = plan_nf()
    order = plan_nf.order.long()           # lane -> row: the waves as the kernel formed them
    torch.cuda.synchronize(dev)
    same = bool(torch.equal(s2, status) and torch.equal(i2, iters) and torch.equal(p2, preds))
    if plan.nfev is not None:              # nfev binning: the timed plan's own waves (its order, its counts)
        order, nf_row = plan.order.long(), plan.nfev
    nf = nf_row[order]
    K = torch.clamp(sl[order].to(torch.int64) - 5, min=0, max=T - 1)
    # SIMT divergence of the refinement: a wave runs until its slowest lane's last scan, each scan as long as its
    # longest lane's window -- wave cost ~ max(nfev) x max(K) over its 64 lanes against the rows' own nfev x K
    nfk = nf.to(torch.int64).cpu().numpy()
    kk = K.cpu().numpy()
    nw = (N + 63) // 64
    pad = nw * 64 - N
    nfw = np.concatenate([nfk, np.zeros(pad, np.int64)]).reshape(nw, 64)
    kw = np.concatenate([kk, np.zeros(pad, np.int64)]).reshape(nw, 64)
    divergence = {"row_scan_steps": int((nfk * kk).sum()),
                  "wave_scan_steps_max_nfev_x_max_K": int((nfw.max(1) * kw.max(1)).sum() * 64),
                  "mean_nfev": float(nfk.mean()), "mean_wave_max_nfev": float(nfw.max(1).mean()),
                  "mean_K": float(kk.mean()), "mean_wave_max_K": float(kw.max(1).mean())}
    divergence["ratio"] = divergence["wave_scan_steps_max_nfev_x_max_K"] / max(1, divergence["row_scan_steps"])
    A_, SUB = 2, 5
    per_step = SUB * (4 * A_ + 7) + 4 * A_ + 5     # Euler sub-steps with the A x 2 sensitivities + residual/gradient
    refine_flop = float((nf.to(torch.int64) * K).sum().item()) * per_step
    final_flop = float(N) * T * SUB * 4            # the refined model's final Euler scan over the whole row
    flop = refine_flop + final_flop
    # V read + int8 arms read + predictions written, statics + seq_len + lane order read, coefficients + status +
    # iterations written
    kbytes = N * T * (8 + 1 + 8) + N * (8 * 2 + 4 + 4) + N * (2 * coh.lib.n_terms * 8 + 8)
    out = {
        "metric": METRIC, "value": N / (ms_step * 1e-3), "unit": "patient-trajectories/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: on-device EQ_4_C cohort, T=60, seq_len U{1..59}, arm flip at a random step",
        "config": {"workload": f"INSITE refinement (BFGS per row, tau=5, lam=10) + Euler-5 rollout, "
                               f"{N // 1000}k rows", "rows": N, "T": T},
        "insite": {"refined_rows": int((st >= 0).sum()), "converged": int((st == 0).sum()),
                   "zoom_failed_fallback": int((st == 3).sum()), "mean_bfgs_iterations": float(it[st >= 0].mean()),
                   "lane_order": ("rows binned by seq_len (device counting sort)" if args.insite_order == "seq_len"
                                  else "rows binned by seq_len (32 levels) and then by the evaluation counts the "
                                       "previous step left (min(nfev, 31); one device counting sort over the "
                                       "combined key)") +
                                 "; the kernel gathers its lanes' patient-major rows through its LDS ring and stores "
                                 "the predictions as row segments (insite_refine_rows_f64; ops.plan_insite_refine, "
                                 "no host sync)",
                   "lane_order_key": args.insite_order,
                   "plan_equals_eager": plan_eq,
                   "identity_lane_order_ms_per_step": ms_identity,
                   "reference_wall_time_s": "88.96 s per INSITE EQ_4_A run incl. 59,000 + 11,800 refinements "
                                            "(results/2_main_table/final_with_insite.txt:2346; SURVEY.md §6)",
                   "mean_evaluations_per_refined_row": float(nf_row.to(torch.float64)[s2 >= 0].mean().item()),
                   "evaluation_count_route_matches": same, "divergence": divergence,
                   "prepare_route_ms_per_step": ms_prepare, "prepare_route_equal": prep_eq},
        "roofline": {"kernel": "insite_refine_kernel<3, 2, 1, WIN, PM> (per-row BFGS + final Euler-5 scan on the "
                               "patient-major rows)", "bound": "valu-f64",
                     "unit": "TFLOP/s", "achieved": flop / (kern_ms * 1e-3) / 1e12, "peak": FP64_VALU_PEAK_TFLOPS,
                     "frac": flop / (kern_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS,
                     "traffic": traffic_for("insite", "insite_refine_kernel<3, 2, 1, true, true>", args=args),
                     "avg_launch_ms": kern_ms,
                     "algorithmic_flop": flop, "flop_per_sensitivity_step": per_step,
                     "flop_method": "sum over refined rows of nfev_r x K_r (K_r = min(seq_len - tau, T - 1)) x "
                                    "(5 Euler sub-steps x (4A + 7) + 4A + 5) with A = 2 arms, + N x T x 5 x 4 for "
                                    "the final scan; nfev from the kernel's own count (insite_refine_general_f64).  The reference's "
                                    "sub-step work: the kernel evaluates the objective scans' sub-steps in closed form "
                                    "(INSITE_REFINE_CF, one FMA per value and step), so this is work done per second "
                                    "in the reference's terms, not executed instructions",
                     "algorithmic_bytes": kbytes, "achieved_GBps": kbytes / (kern_ms * 1e-3) / 1e9,
                     "avg_ms_source": "HIP events on the launch stream around args.steps back-to-back launches of "
                                      "insite_refine_rows_f64 with the step's lane order (the sort excluded)"},
    }
    # the same kernel in EXECUTED terms: instruction counters, and the bytes the kernel streams as executed -- every
    # objective scan of a wave refills its LDS ring for all 64 rows up to the wave's longest window, in 8-step slots,
    # as long as any lane has a trial pending (wave max nfev x slots(wave max K + 1) x 64 rows x 8 B), plus the final
    # scan's V + arms read and the predictions written -- against the measured traffic
    ex = pmc_executed("profiles/r05/refine_pmc_scan/summary.json", "insite_refine_kernel<3, 2, 1, true, true>",
                      args=args, config="insite")
    if ex is not None:
        ring_b = float((nfw.max(1) * ((kw.max(1) + 1 + 7) // 8 * 8)).sum()) * 64 * 8
        ex["executed_ring_read_bytes"] = ring_b
        ex["row_window_read_bytes"] = float((nf.to(torch.int64) * (K + 1)).sum().item()) * 8
        ex["final_scan_bytes"] = float(N * T * (8 + 1 + 8))
        if "fetch_bytes_raw" in ex:
            # two calibrations bracket this shape (the ring's DMA moves 64-B runs of 16 rows per instruction):
            # wide streaming (FETCH_SIZE = 1/2 of the bytes) and C5's 64-B per-row runs (0.617, profiles/r05/c5cal)
            exe = ring_b + N * T * (8 + 1)
            ex["fetch_over_executed_reads_x2"] = ex["fetch_bytes_x2"] / exe
            ex["fetch_over_executed_reads_runcal"] = ex["fetch_bytes_raw"] / 0.617 / exe
        out["roofline"]["executed"] = ex
    if not args.no_parity:
        o_ = plan.order.long()
        out["parity"] = insite_parity(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, preds, coef, status, iters,
                                      extra=(o_[:64].cpu().numpy(), o_[-64:].cpu().numpy()))
        # the literal reading of sindy.py:628-631 (status 3 reverts to the global model): the same
        # rows through the product call with revert_on_zoom_fail and the oracle with the same flag (untimed)
        rplan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, revert_on_zoom_fail=True)
        rp, rc, rs_, ri = (t.clone() for t in rplan())
        out["parity_revert_mode"] = insite_parity(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, rp, rc, rs_, ri,
                                                  extra=(o_[:64].cpu().numpy(), o_[-64:].cpu().numpy()), revert=True)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    emit(out)


# planted per-arm model of the F4 cohort over [1, x0, u0, x0 u0]: no treatment / chemo / radio / both
F4_COEF = [[0.0, 0.20, 0.0, 0.0], [0.0, 0.0, 0.0, -0.60], [0.0, -0.30, 0.0, 0.0], [0.0, -0.25, 0.0, -0.90]]


def _insite4_rows(N, T, seed, device):
    """The INSITE4 rows (cancer_sim / EQ_5 shape): F4's 4-arm cohort (planted per-arm model, Markov arms, Euler-5
    truth + 0.01 noise) patient-major, arm index = treatment code (chemo | radio << 1), seq_len U{1..59}."""
    from insite_amd import cohort
    coh = cohort.synthetic_segments(N, T, seed=seed, device=device, coef=F4_COEF, dt=0.1)
    g = torch.Generator(device=device)
    g.manual_seed(seed + 1)
    sl = torch.randint(1, T, (N,), generator=g, device=device, dtype=torch.int32)
    return coh.x[:T, :N].t().contiguous(), coh.arm[:, :N].t().contiguous(), coh.u, sl, coh.lib, coh.dt


def _insite4_models(V, arm, u, dt, lib, n_fit=20_000):
    """The three global models the 4-arm INSITE line refines: (1) ``sparse`` = the planted per-arm model scaled by
    1.1 (5 active terms: every row has something to refine), (2) ``dense`` = (1) with the 11 zero terms at 0.01 --
    all 16 active, as the reference's cancer_sim model (final_with_insite.txt:2326 logs 16 non-zero terms), and
    (3) ``joint`` = the one-ODE model over [x0, chemo, radio, u0] (sindy.py:503-517) least-squares fitted to forward
    differences of the first ``n_fit`` rows, |c| <= 1e-3 dropped."""
    from insite_amd.library import polynomial_library
    base = np.array(F4_COEF) * 1.1
    lib_j = polynomial_library(1, 2, True, n_inputs=2)
    n = min(n_fit, V.size(0))
    x = V[:n].cpu().numpy()
    a = arm[:n].cpu().numpy().astype(np.int64)
    uu = u[:n, 0].cpu().numpy()
    T = x.shape[1]
    cols = np.stack([x[:, :-1], (a[:, :-1] & 1).astype(np.float64), ((a[:, :-1] >> 1) & 1).astype(np.float64),
                     np.repeat(uu[:, None], T - 1, axis=1)], axis=-1).reshape(-1, 4)
    ex = lib_j.exps.astype(np.int64)
    theta = np.prod(cols[:, None, :] ** ex[None, :, :], axis=2)
    xd = ((x[:, 1:] - x[:, :-1]) / dt).reshape(-1)
    cj = np.linalg.lstsq(theta, xd, rcond=None)[0]
    cj[np.abs(cj) <= 1e-3] = 0.0
    return {"sparse": (base, lib), "dense": (np.where(base != 0, base, 0.01), lib), "joint": (cj[None, :], lib_j)}


def _insite4_rows_np(N, T, seed, dt=0.1, switch_p=0.1, noise=0.01):
    """Host rows of the same distribution as _insite4_rows (numpy; for the CPU leg, drawn before any GPU context):
    u ~ N(0.5, 0.05), y0 ~ U(1, 5), Markov arms over 4 codes (switch 0.1 per step), Euler-5 of F4's model."""
    rng = np.random.default_rng(seed)
    c = np.array(F4_COEF)
    u = rng.normal(0.5, 0.05, (N, 1))
    y = rng.uniform(1.0, 5.0, N)
    arm = np.empty((N, T), dtype=np.int8)
    cur = rng.integers(0, 4, N)
    x = np.empty((N, T + 1))
    x[:, 0] = y
    h = dt / 5.0
    for k in range(T):
        arm[:, k] = cur
        ca = c[cur]
        for _ in range(5):
            y = y + h * (ca[:, 0] + ca[:, 1] * y + ca[:, 2] * u[:, 0] + ca[:, 3] * y * u[:, 0])
        x[:, k + 1] = y
        sw = rng.random(N) < switch_p
        cur = np.where(sw, rng.integers(0, 4, N), cur)
    x += noise * rng.normal(size=x.shape)
    sl = rng.integers(1, T, N).astype(np.int32)
    return x[:, :T], arm, u, sl


def _cpu_refine4_chunk(bounds):
    from oracle import insite_refine_ref as Q
    lo, hi = bounds
    d = _CPU
    for i in range(lo, hi):
        Q.refine_patient(d["V"][i], d["arm"][i], d["u"][i], int(d["sl"][i]), d["c0"], d["ex"], d["dt"], 10.0, 5)
    return hi - lo


def insite4_cpu_baseline(V, arm, u, sl, c0, ex, dt, per_worker=256):
    """Bounded CPU sample of the 4-arm dense INSITE workload: the oracle's restatement of the jax BFGS refinement
    (oracle/insite_refine_ref.py) on up to per_worker x workers host rows of the benched distribution
    (_insite4_rows_np), over the host's workers (a forked pool: call before the GPU context exists)."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    info = host_info()
    W = info["workers"]
    n = min(W * per_worker, V.shape[0])
    _CPU.update(V=V[:n], arm=arm[:n], u=u[:n], sl=sl[:n], c0=c0, ex=ex, dt=dt)
    chunks = [(int(a[0]), int(a[-1]) + 1) for a in np.array_split(np.arange(n), W) if a.size]
    with worker_pool(mp.get_context("fork"), W, _cpu_worker_init) as pool:
        pool.map(abs, range(W))
        t0 = time.perf_counter()
        pool.map(_cpu_refine4_chunk, chunks)
        el = time.perf_counter() - t0
    for k in ("V", "arm", "u", "sl"):
        _CPU.pop(k, None)
    return {"value": n / el, "unit": "patient-trajectories/s", "cores": W, "kind": "port",
            "sample": f"oracle/insite_refine_ref.py (jax BFGS restated, numpy) on {n} host rows of the benched "
                      f"4-arm distribution (T = 60, seq_len U{{1..59}}) with the dense model (16 active coefficients) "
                      f"over a {W}-process pool, {el:.2f} s", "host": info}


def insite4_main(args):
    """INSITE refinement of the 4-arm models (the cancer_sim / EQ_5 path, sindy.py:484-551; the reference's slowest
    published path, cancer_sim INSITE 83.5 s, final_with_insite.txt:2326): 1M rows x T = 60 with int8 per-step arms
    0..3, one static, tau = 5, lam = 10 (config/config.yaml:24-27).  Three global models: sparse per-arm (5 active
    terms, the register-resident M = 8 kernel), dense per-arm (16 active, the M = 16 kernel -- the line's value,
    as the reference's cancer_sim model is dense) and the joint one-ODE model (insite_refine_general_f64's folded
    treatment combinations).  One step = one refinement of every row: the seq_len sort, the gather pass, the kernel
    and the scatter pass (ops.plan_insite_refine, 4 C calls)."""
    from insite_amd import ops
    N = args.patients if args.patients != 100_000 else 1_000_000
    T = 60
    cpu = None
    if not args.no_cpu_baseline:   # host rows first (no GPU context yet: the pool forks)
        from insite_amd.library import polynomial_library
        Vc, ac, uc, slc = _insite4_rows_np(4096, T, args.seed + 41)
        c_dense = np.where(np.array(F4_COEF) != 0, np.array(F4_COEF) * 1.1, 0.01)
        cpu = insite4_cpu_baseline(Vc, ac, uc, slc, c_dense, polynomial_library(1, 2, True).exps.astype(np.int64), 0.1)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    V, arm, u, sl, lib, dt = _insite4_rows(N, T, args.seed + 41, dev)
    models = _insite4_models(V, arm, u, dt, lib)
    st_ = torch.cuda.current_stream(dev)
    res = {}
    for name, (c0, lb) in models.items():
        plan = ops.plan_insite_refine(V, arm, u, sl, c0, lb, dt, 10.0, 5, order=args.insite_order)
        for _ in range(args.warmup):
            plan()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            preds, coef, status, iters = plan()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        kidx = plan.kernel_call                  # [(key,) sort, prepare, kernel, finish(, nfev scatter)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st_)
        for _ in range(args.steps):
            plan.call(kidx, st_)
        e1.record(st_)
        torch.cuda.synchronize(dev)
        kern_ms = e0.elapsed_time(e1) / args.steps
        nf = torch.empty((N,), dtype=torch.int32, device=dev)
        p2, _, s2, _ = ops.insite_refine(V, arm, u, sl, c0, lb, dt, 10.0, 5, nfev=nf)
        torch.cuda.synchronize(dev)
        K = torch.clamp(sl.to(torch.int64) - 5, min=0, max=T - 1)
        A_, SUB = 4, 5
        per_step = SUB * (4 * A_ + 7) + 4 * A_ + 5
        flop = float((nf.to(torch.int64) * K).sum().item()) * per_step + float(N) * T * SUB * 4
        stn = status.cpu().numpy()
        m_act = int((np.abs(c0) > 1e-3).sum())
        res[name] = {"active_coefficients": m_act, "ms_per_step": ms, "kernel_ms": kern_ms,
                     "lane_order_key": args.insite_order,
                     "kernel": ("insite_refine_coop_kernel<16, 4>" if 8 < m_act <= 16 and os.environ.get("INSITE_REFINE_COOP", "1") != "0"
                                else f"insite_refine_kernel<{2 if m_act <= 2 else 3 if m_act == 3 else 4 if m_act <= 4 else 6 if m_act <= 6 else 8 if m_act <= 8 else 16 if m_act <= 16 else 36}, 4, 1>"),
                     "valu_f64_TFLOPs": flop / (kern_ms * 1e-3) / 1e12,
                     "frac": flop / (kern_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS,
                     "refined_rows": int((stn >= 0).sum()), "converged": int((stn == 0).sum()),
                     "mean_bfgs_iterations": float(iters.cpu().numpy()[stn >= 0].mean()),
                     "mean_evaluations_per_refined_row": float(nf.to(torch.float64)[s2 >= 0].mean().item()),
                     "equal_to_nfev_route": bool(torch.equal(p2, preds) and torch.equal(s2, status)),
                     "finite_predictions": bool(torch.isfinite(preds).all().item()), "algorithmic_flop": flop}
        # evaluation-count divergence inside a wave: a wave runs as many objective scans as its slowest row
        # (8 rows a wave in the cooperative kernel, 64 in the one-row-per-lane kernels), rows in the lane order
        o_ = plan.order.long() if getattr(plan, "order", None) is not None else torch.arange(N, device=dev)
        rpw = 8 if res[name]["kernel"].startswith("insite_refine_coop") else 64
        nfo = nf.index_select(0, o_).to(torch.float64)
        nfo = torch.cat([nfo, nfo.new_zeros((-N) % rpw)]).view(-1, rpw)
        res[name]["wave_divergence"] = {"rows_per_wave": rpw, "max_over_mean_evaluations":
                                        float(nfo.max(1).values.sum().item() * rpw / max(nfo.sum().item(), 1.0))}
        if not args.no_parity:   # the dense / joint oracle rows cost ~4 ms each on one host core
            res[name]["parity"] = insite_parity(V, arm, u, sl, c0, lb, dt, 10.0, 5, preds, coef, status, iters,
                                                n_sample=4096 if name == "sparse" else 2048, seed=17,
                                                extra=(o_[:64].cpu().numpy(), o_[-64:].cpu().numpy()))
    d = res["dense"]
    kb = N * T * (8 + 1 + 8) + N * (8 + 4) + N * (16 * 8 + 8)
    out = {
        "metric": METRIC, "value": N / (d["ms_per_step"] * 1e-3), "unit": "patient-trajectories/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": d["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: on-device 4-arm cohort (F4's planted model, Markov arms, Euler-5 truth + 0.01 noise), "
                "T=60, seq_len U{1..59}",
        "config": {"workload": f"INSITE refinement, 4 arms (cancer_sim / EQ_5 path; BFGS per row, tau=5, lam=10) + "
                               f"Euler-5 rollout, {N // 1000}k rows; value = the dense per-arm model", "rows": N,
                   "T": T, "arms": 4},
        "models": res,
        "roofline": {"kernel": d["kernel"] + " (dense per-arm model: 8 lanes per row, H rows in VGPRs)",
                     "bound": "valu-f64", "unit": "TFLOP/s", "achieved": d["valu_f64_TFLOPs"],
                     "peak": FP64_VALU_PEAK_TFLOPS, "frac": d["frac"],
                     "traffic": traffic_for("insite4", d["kernel"].split("<")[0] + "<16, 4", args=args),
                     "avg_launch_ms": d["kernel_ms"], "algorithmic_flop": d["algorithmic_flop"],
                     "flop_method": "sum over refined rows of nfev_r x K_r x (5 x (4A + 7) + 4A + 5), A = 4 arms, + N x T "
                                    "x 5 x 4 for the final scan; nfev from the kernel's own count (the reference's sub-step work; "
                                    "the objective scans run it in closed form, INSITE_REFINE_CF)",
                     "algorithmic_bytes": kb, "achieved_GBps": kb / (d["kernel_ms"] * 1e-3) / 1e9},
    }
    ex = pmc_executed("profiles/r05/coop_pmc2/summary.json", "insite_refine_coop_kernel<16, 4, true>")
    if ex is not None and N == 1_000_000:
        ex["note"] = "counters averaged over the dense and joint models' launches (16 dispatches)"
        out["roofline"]["executed"] = ex
    if "parity" in d:
        out["parity"] = dict(d["parity"], model="dense (the line's value); every model's in models.*.parity")
    if cpu is not None:
        out["cpu_baseline"] = cpu
    emit(out)


def f4_main(args):
    """Treatment-segment path of the cancer_sim / EQ_5 datasets (reference
    pkpd/utils.py:433-462, 607-637, sindy.py:193-216, 289-312): 1M patients x 60 steps, 4 arms, one
    static.  One step = discovery (segment split + FD order 1 + library + per-arm Gram in one kernel,
    fixed-order reduction fused with the four STLSQ fits) + Euler-5 (the reference odeint) 4-arm
    counterfactual rollout under fresh per-step arms."""
    from insite_amd import ops, cohort
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N = args.patients if args.patients != 100_000 else 1_000_000
    T = args.T if args.T != 200 else 60
    coh = cohort.synthetic_segments(N, T, seed=args.seed + 31, device=dev, coef=F4_COEF, dt=0.1)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 32)
    arm_cf = cohort.markov_arms(N, T, 4, 0.1, g, dev)
    lib, F = coh.lib, coh.lib.n_terms
    out = (torch.empty((4, F), dtype=torch.float64, device=dev), torch.empty((4, F), dtype=torch.int8, device=dev),
           torch.empty((4,), dtype=torch.int32, device=dev), torch.empty((4, F, F), dtype=torch.float64, device=dev),
           torch.empty((4, F), dtype=torch.float64, device=dev))
    y = torch.empty((T, N), dtype=torch.float64, device=dev)
    y0 = coh.x[0].contiguous()
    ws = ops.Workspace()
    fit = ops.plan_sindy_fit_segments(coh.x, coh.arm, coh.seq_len, coh.u, coh.dt, lib, 0.001, 0.5, workspace=ws,
                                      out=out, layout="time")
    roll = ops.plan_rollout(y0, coh.u, arm_cf, out[0], lib, coh.dt, method="euler5", T=T, out=y, layout="time")
    gram = ops.plan_gram_segments(coh.x, coh.arm, coh.seq_len, coh.u, coh.dt, lib, 4, "order1", ws,
                                  out=(out[3], out[4]), layout="time")

    def step(st):
        fit(st)
        roll(st)

    st = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        step(st)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(st)
    torch.cuda.synchronize(dev)
    ms_step = (time.perf_counter() - t0) / args.steps * 1e3

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            fn(st)
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    n_roof = max(args.steps, 10)
    gram_ms = timed(gram, n_roof)
    roll_ms = timed(roll, n_roof)
    gb = N * (T + 1) * 8 + N * T + N * (8 * lib.n_statics + 4)          # x samples + arms + (u, seq_len)
    rb = rollout_bytes(N, T, U=lib.n_statics)
    achieved = gb / (gram_ms * 1e-3) / 1e9
    res = {
        "metric": METRIC, "value": N / (ms_step * 1e-3), "unit": "patient-trajectories/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: on-device 4-arm cohort (planted per-arm model, Markov arms p=0.1, Euler-5 truth + 0.01 noise)",
        "config": {"workload": f"F4: cancer_sim/EQ_5 path, {N // 1000}k patients x {T} steps, 4 arms: segment-split "
                               f"FD1 discovery + STLSQ (threshold 0.001) + Euler-5 4-arm counterfactual rollout",
                   "patients": N, "T": T, "arms": 4, "library_terms": F,
                   "discovered_support": (out[1].cpu().numpy() != 0).astype(int).tolist(),
                   # recovery check of the planted model: with the reference's cancer_sim / EQ_5 threshold
                   # (0.001, config/config.yaml:20-23) the first-order FD bias and the 0.01 observation noise
                   # leave small spurious terms above the threshold — reported, not hidden
                   "planted_support": (np.array(F4_COEF) != 0).astype(int).tolist(),
                   "support_equals_planted": bool(np.array_equal(out[1].cpu().numpy() != 0, np.array(F4_COEF) != 0)),
                   "planted_terms_recovered": bool(np.all((out[1].cpu().numpy() != 0)[np.array(F4_COEF) != 0])),
                   "max_abs_coef_error_vs_planted": float(np.max(np.abs(out[0].cpu().numpy() - np.array(F4_COEF)))),
                   "max_abs_spurious_coef": float(np.max(np.abs(np.where(np.array(F4_COEF) != 0, 0.0,
                                                                         out[0].cpu().numpy())))),
                   "support_note": "exact planted-support recovery is not expected at the reference's threshold "
                                   "(0.001): with FiniteDifference(order=1) per treatment segment the backward "
                                   "difference closing a segment is a different affine relation in x than the "
                                   "interior forward differences, so the least-squares fit blends them into small "
                                   "spurious terms even on noise-free data (the reference algorithm's own output: "
                                   "tests/test_gpu_segments.py pins the GPU support to the oracle restatement)"},
        "roofline": {"kernel": "gram_seg_kernel (order1, 4 arms; in-launch fixed-order reduction, G|b written by the "
                               "last block)", "bound": "hbm",
                     "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic_for("f4", "gram_seg_kernel", args=args), "algorithmic_bytes_per_launch": gb,
                     "avg_launch_ms": gram_ms},
        "rollout": {"kernel": "rollout_tm_kernel (euler5, 4 arms, int8 arms)", "avg_launch_ms": roll_ms,
                    "algorithmic_bytes": rb, "achieved_GBps": rb / (roll_ms * 1e-3) / 1e9,
                    "frac": rb / (roll_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS},
    }
    if not args.no_parity:
        res["parity"] = f4_parity(coh, arm_cf, lib, T, out[0], out[1], y)
    if not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import insite_ref as R
        from oracle import segments_ref as S
        n_s = min(10 * args.cpu_sample, N)         # ~10 s of one host core at the default sizes
        xs = coh.x[:, :n_s].T.contiguous().cpu().numpy()
        us = coh.u[:n_s].cpu().numpy()
        a_f = coh.arm[:, :n_s].T.cpu().numpy().astype(np.int64)
        a_c = arm_cf[:, :n_s].T.cpu().numpy().astype(np.int64)
        sl = np.full(n_s, T, dtype=np.int64)
        ex = lib.exps.astype(np.int64)
        # the host's workers as threads over patient chunks (the vectorised numpy kernels release the GIL;
        # a forked pool is not safe once this process holds a GPU context), one BLAS thread each
        from concurrent.futures import ThreadPoolExecutor
        info = host_info()
        W = info["workers"]
        parts = [(int(q[0]), int(q[-1]) + 1) for q in np.array_split(np.arange(n_s), W) if q.size]
        try:
            from threadpoolctl import threadpool_limits
            lim = threadpool_limits(limits=1)
        except Exception:  # pragma: no cover
            lim = None
        with ThreadPoolExecutor(W) as ex_pool:
            list(ex_pool.map(lambda q: q, range(W)))
            t1 = time.perf_counter()
            gb_parts = list(ex_pool.map(lambda q: S.gram_segments_vectorized(xs[q[0]:q[1]], us[q[0]:q[1]],
                                                                                a_f[q[0]:q[1]], sl[q[0]:q[1]], coh.dt, ex),
                                        parts))
            G = sum(g_[0] for g_ in gb_parts)
            b = sum(g_[1] for g_ in gb_parts)
            c = np.stack([R.stlsq_gram(G[k], b[k], 0.001, 0.5)[0] for k in range(4)])
            list(ex_pool.map(lambda q: R.rollout(xs[q[0]:q[1], 0], us[q[0]:q[1]], a_c[q[0]:q[1]], c, ex, coh.dt,
                                                 method="euler5"), parts))
            el = time.perf_counter() - t1
        del lim
        res["cpu_baseline"] = {"value": n_s / el, "unit": "patient-trajectories/s", "cores": W, "kind": "port",
                               "sample": f"oracle/segments_ref.py + insite_ref.rollout (numpy, vectorised over patients) "
                                         f"on {n_s} patients x {T} steps over {W} threads (patient chunks), {el:.2f} s",
                               "host": info}
    emit(res)


def c4_main(args):
    """Configuration C4 (BASELINE.json configs[3]): PK/PD EQ_4_C, 1M patients, heterogeneous per-patient
    coefficients.  One step = global discovery (Gram [-> RCCL all-reduce of G|b when N > 1] -> STLSQ),
    per-patient STLSQ from the global support (LSQIntialMask, pkpd_simulation.py:791-800; moments pass +
    one fit per patient), then the per-patient-coefficient Euler-5 counterfactual rollout
    (predict_with_reduced_coefs, sindy.py:767-778).  Patients shard contiguously over ranks
    (N_total / world per rank: strong scaling, as configs[3] fixes 1M patients on 8 GPUs)."""
    from insite_amd import ops, cohort
    from insite_amd import dist as idist
    world, rank, dev = dist_setup()
    N_total = args.patients if args.patients != 100_000 else 1_000_000
    T = args.T if args.T != 200 else 60
    lo, hi = idist.shard_bounds(N_total, rank, world)
    N = hi - lo
    coh = cohort.synthetic_pkpd(N, T, seed=args.seed * 1000 + 3 + rank, device=dev, equation="EQ_4_C", layout="time")
    arm_cf = cohort.counterfactual_arms(coh.arm, T, seed=args.seed * 1000 + 3 + rank, layout=bits_layout(args.arm_format))
    lib, F = coh.lib, coh.lib.n_terms
    buf = idist.MomentBuffer(2, F, dev)
    gout = (torch.empty((2, F), dtype=torch.float64, device=dev), torch.empty((2, F), dtype=torch.int8, device=dev),
            torch.empty((2,), dtype=torch.int32, device=dev))
    pout = (torch.empty((N, 2, F), dtype=torch.float64, device=dev), torch.empty((N, F), dtype=torch.int8, device=dev),
            torch.empty((N,), dtype=torch.int32, device=dev))
    y = torch.empty((T, N), dtype=torch.float64, device=dev)
    ws, wsp = ops.Workspace(), ops.Workspace()

    mom = torch.empty((N, 5), dtype=torch.float64, device=dev)

    def discover():
        """ONE pass over x gives the Gram and every patient's moments (insite_gram_moments_f64): single rank
        with the global STLSQ fused in; N > 1: all-reduce G|b, then the replicated STLSQ."""
        if world == 1:
            ops.gram_moments(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, workspace=ws,
                             out=(*gout, buf.G, buf.b, mom), layout="time")
        else:
            ops.gram_moments(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, None, workspace=ws,
                             out=(None, None, None, buf.G, buf.b, mom), layout="time")
            idist.reduce_moments(buf)
            ops.stlsq(buf.G, buf.b, 0.1, 0.5, out=gout)

    def per_patient():
        ops.fit_per_patient_moments(mom, coh.u, coh.arm, coh.rows, T, lib, gout[0], 0.1, 0.5, out=pout)

    # the per-patient refit folded into the rollout (insite_refit_rollout_moments_f64): one launch, the
    # per-patient coefficient rows never reach HBM; the two-call form (fit, then per-row rollout) is timed
    # beside it as "two_call_alternative"
    fold = ops.plan_refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, lib, gout[0], 0.1, 0.5, coh.y0, arm_cf,
                                          coh.dt, T, method="euler5", out=y)

    def step():
        discover()
        fold()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = idist.max_over_ranks(time.perf_counter() - t0, dev)
    ms_step = el / args.steps * 1e3
    st = torch.cuda.current_stream(dev)

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(n):
            fn()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    n_roof = max(args.steps, 5)
    disc_ms = timed(discover, n_roof)
    fold_ms = timed(fold, n_roof)
    pp_ms = timed(per_patient, n_roof)
    roll_ms = timed(lambda: ops.rollout(coh.y0, coh.u, arm_cf, pout[0], lib, coh.dt, method="euler5", T=T, out=y,
                                        layout="time_bits"), n_roof)
    # the refits themselves (iterations, supports): one untimed launch with the optional outputs
    ops.refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, lib, gout[0], 0.1, 0.5, coh.y0, arm_cf, coh.dt, T,
                              out=y, fits=pout)
    it = pout[2].to(torch.float64)
    if rank == 0:
        fb = rollout_bytes(N, T, arm_bits=1) + N * (5 * 8 + 1 + 4)      # + moments / factual arm / rows read
        rb = rollout_bytes(N, T, arm_bits=1) + N * 2 * F * 8            # two-call: + the per-patient coefficient rows
        db = N * T * 8 + N * (2 * 8 + 1 + 4) + N * 5 * 8                # x + statics/arm/rows in, moments out
        pb = N * 5 * 8 + N * (2 * 8 + 1 + 4) + N * (2 * F * 8 + F + 4)  # moments + statics/arm/rows in, fits out
        res = {
            "metric": METRIC, "value": N_total / (ms_step * 1e-3), "unit": "patient-trajectories/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: on-device EQ_4_C PK/PD cohort (reference distributions, Euler-5 truth + 0.01 noise)",
            "config": {"workload": f"C4: PK/PD {N_total // 1000}k patients x {T} steps: global discovery and every "
                                   f"patient's moments in one pass (+ RCCL all-reduce when N>1) + per-patient STLSQ "
                                   f"folded into the per-patient-coefficient Euler-5 rollout", "patients_total": N_total, "patients_per_gpu": N, "T": T,
                       "parallelism": f"patient-shard x{world}",
                       "global_support": (gout[1].cpu().numpy() != 0).astype(int).tolist(),
                       "mean_per_patient_iterations": float(it.mean())},
            "roofline": {"kernel": "refit_rollout_kernel (per-patient refit from the moments in the prologue + "
                                   "euler5 bit-arm rollout)", "bound": "hbm",
                         "achieved": fb / (fold_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": fb / (fold_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, "traffic": traffic_for("c4", "refit_rollout_kernel", args=args),
                         "algorithmic_bytes_per_launch": fb, "avg_launch_ms": fold_ms},
            "discovery": {"kernels": "gram_kernel<MOM=2> (Gram + in-launch reduction + STLSQ + every patient's "
                                     "moments, one pass over x)" + (" + RCCL all-reduce + stlsq_kernel" if world > 1 else ""),
                          "avg_ms": disc_ms, "algorithmic_bytes": db, "achieved_GBps": db / (disc_ms * 1e-3) / 1e9},
            "two_call_alternative": {
                "kernels": "patient_fit_kernel<7> (from the moments) + rollout_tm_kernel (per-patient coefficient rows)",
                "per_patient_fit_ms": pp_ms, "per_patient_fit_bytes": pb,
                "per_patient_fit_GBps": pb / (pp_ms * 1e-3) / 1e9, "rollout_ms": roll_ms, "rollout_bytes": rb,
                "rollout_GBps": rb / (roll_ms * 1e-3) / 1e9, "sum_ms": pp_ms + roll_ms},
        }
        if world == 1 and not args.no_parity:
            sys.path.insert(0, ROOT)
            res["parity"] = c4_parity(coh, arm_cf, lib, T, gout[0], gout[1], pout, y)
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, ROOT)
            from oracle import insite_ref as R
            n_s = min(200_000, N)                      # ~12 s of host-core work
            xs = coh.x[:T, :n_s].T.contiguous().cpu().numpy()
            us, ar, rw = coh.u[:n_s].cpu().numpy(), coh.arm[:n_s].cpu().numpy(), coh.rows[:n_s].cpu().numpy()
            gc = gout[0].cpu().numpy()
            # a per-patient Python loop: a SPAWNED process pool (fork is not safe once this process holds a
            # GPU context; spawn starts fresh interpreters that never touch the GPU)
            import multiprocessing as mp
            info = host_info()
            W = info["workers"]
            ex = lib.exps.astype(np.int64)
            chunks = [(int(q[0]), int(q[-1]) + 1) for q in np.array_split(np.arange(n_s), W) if q.size]
            # the sample travels to the workers at start-up (initargs), outside the clock
            with worker_pool(mp.get_context("spawn"), W, _cpu_pp_init, (xs, us, ar, rw, coh.dt, ex, gc)) as pool:
                pool.map(abs, range(W))
                t1 = time.perf_counter()
                pool.map(_cpu_pp_fit_chunk, chunks)
                el1 = time.perf_counter() - t1
            res["cpu_baseline"] = {"value": n_s / el1, "unit": "patients/s (per-patient STLSQ only)", "cores": W,
                                   "kind": "port", "sample": f"oracle/insite_ref.per_patient_fit (row-form pysindy-style "
                                                            f"STLSQ per patient) on {n_s} patients over a {W}-process "
                                                            f"spawned pool, {el1:.2f} s", "host": info}
        emit(res)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(args):
    """``--gpus N`` (N > 1) without a torch.distributed environment: start N ranks (one per GPU) through
    torchrun as a CHILD process — before anything touches the GPU — and exit with its status.  Inside a
    distributed launch, WORLD_SIZE must equal --gpus (exit 2 otherwise)."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus <= 1:
            return
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))
    if int(world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a mislabelled run",
              file=sys.stderr)
        sys.exit(2)


def dist_setup(force_group: bool = False):
    """(world, rank, device) of this process; joins the process group when world > 1 (or, with
    ``force_group``, as a single-rank RCCL group: --force-collective).  Rehearsal knobs for a one-GPU box
    (never set by the driver): INSITE_REHEARSE_ONE_GPU puts every rank on cuda:0 and INSITE_DIST_BACKEND=gloo
    swaps RCCL for gloo."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if os.environ.get("INSITE_REHEARSE_ONE_GPU") else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or force_group:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        backend = os.environ.get("INSITE_DIST_BACKEND", "nccl")
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))
    return world, rank, dev


TRAFFIC_R04 = os.path.join(ROOT, "profiles", "traffic_r04.json")
TRAFFIC_R05 = os.path.join(ROOT, "profiles", "traffic_r05.json")
TRAFFIC_R06 = os.path.join(ROOT, "profiles", "traffic_r06.json")


def traffic_for(config, kernel, grid=None, args=None):
    """HBM bytes per launch of `kernel` (symbol prefix) in the bench line `config`, from the committed PMC passes
    (profiles/traffic_r05.json, else traffic_r04.json; tools/g_traffic.sh + tools/traffic_summary.py: FETCH_SIZE x 2 +
    WRITE_SIZE, median per dispatch), or None when that table has no such entry.  `grid`: the launch's total
    threads when a config launches the kernel at several sizes.  `args`: the table was taken on each config's
    DEFAULT workload at N = 1 (tools/g_traffic.sh), so a line with other sizes gets None."""
    if args is not None:   # exactly the workload the table was taken on, or nothing
        # the configs' sentinels: --patients 100000 means 1M for every config but c2, --T 200 means 500 (c3) or
        # 60 (c4, f4); compare the EFFECTIVE sizes, so an explicit --T 60 on c4 is its default workload too
        big = config != "c2"
        eff_n = 1_000_000 if (big and args.patients == 100_000) else args.patients
        t_def = {"c3": 500, "c4": 60, "f4": 60, "ns": 500}.get(config, 200)
        eff_t = t_def if args.T == 200 else args.T
        # the north-star step reads its arms in the --ns-arms format (default tile-major bits), the others --arm-format
        fmt, fmt_def = (args.ns_arms, "tiles") if config == "ns" else (args.arm_format, "bits")
        knobs = (eff_n, eff_t, args.method, fmt, args.layout, args.gram_blocks, args.dstreams,
                 int(os.environ.get("WORLD_SIZE", "1")))
        if knobs != (1_000_000 if big else 100_000, t_def, "rk4", fmt_def, "time", 0, 1, 1):
            return None
    # this round's table first (taken on the kernels as they are now), the previous round's for configs it lacks
    hits = []
    for path in (TRAFFIC_R06, TRAFFIC_R05, TRAFFIC_R04):
        try:
            with open(path) as f:
                tab = json.load(f).get(config, {})
        except Exception:
            continue
        hits = [v for v in tab.values() if v.get("kernel", "").startswith(kernel)
                and (grid is None or str(v.get("grid_size")) == str(grid))]
        if hits:
            break
    if not hits:
        return None
    best = max(hits, key=lambda v: v.get("dispatches") or 0)
    return best.get("hbm_bytes")


def pmc_executed(path, kernel, args=None, config=None):
    """Executed-instruction view of one kernel from a committed rocprofv3 --pmc summary (tools/pmc_summary.py of
    tools/g_r05_refine_pmc.sh passes, taken on the line's default workload): VALU instructions per launch and
    their share of the SIMD cycles (SQ_INSTS_VALU x 4 cycles over 1024 SIMDs x the kernel's cycles, SQ_BUSY_CYCLES /
    32 shader engines), SALU / LDS / vector-memory instruction counts, FETCH_SIZE (x2: wide-streaming calibration)
    and WRITE_SIZE bytes.  None when the summary is absent or the line runs a non-default workload."""
    if args is not None and config is not None and traffic_for(config, kernel, args=args) is None:
        return None
    try:
        with open(os.path.join(ROOT, path)) as f:
            d = json.load(f)
    except Exception:
        return None
    v = {}
    for run in d.values():
        for k, x in run.items():
            if k.startswith(kernel):
                v[k.split()[-1]] = x["mean"]
    if "SQ_INSTS_VALU" not in v or "SQ_BUSY_CYCLES" not in v:
        return None
    cyc = v["SQ_BUSY_CYCLES"] / 32.0
    out = {"pmc_source": path, "kernel_cycles": cyc, "valu_instructions": v["SQ_INSTS_VALU"],
           "valu_busy_frac": v["SQ_INSTS_VALU"] * 4.0 / (1024.0 * cyc),
           "salu_instructions": v.get("SQ_INSTS_SALU"), "lds_instructions": v.get("SQ_INSTS_LDS"),
           "vmem_read_instructions": v.get("SQ_INSTS_VMEM_RD"), "waves": v.get("SQ_WAVES")}
    if "FETCH_SIZE" in v:
        out["fetch_bytes_raw"] = v["FETCH_SIZE"] * 1024
        out["fetch_bytes_x2"] = v["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in v:
        out["write_bytes"] = v["WRITE_SIZE"] * 1024
    return out


def c5_traffic_calibrated(args):
    """The RK45 kernel's HBM bytes per launch with its own access shape's calibration (window refills: FETCH_SIZE
    reports 0.617 of the bytes; 64-B sector writes: WRITE_SIZE 1.081; tools/probe/window_probe.hip), from the
    committed counters of the default C5 workload, or None."""
    if traffic_for("c5", "rollout_rk45_flat_kernel", args=args) is None:
        return None
    try:
        with open(os.path.join(ROOT, "profiles", "r05", "c5cal", "calibration.json")) as f:
            cal = json.load(f)
    except Exception:
        return None
    hits = []
    for path in (TRAFFIC_R06, TRAFFIC_R05, TRAFFIC_R04):
        try:
            with open(path) as f:
                tab = json.load(f).get("c5", {})
        except Exception:
            continue
        hits = [v for v in tab.values() if v.get("kernel", "").startswith("rollout_rk45_flat_kernel")]
        if hits:
            break
    if not hits:
        return None
    v = max(hits, key=lambda v: v.get("dispatches") or 0)
    return (v["FETCH_SIZE_KiB_median"] * 1024 / cal["fetch_factor"]
            + v["WRITE_SIZE_KiB_median"] * 1024 / cal["write_factor"])


def step_traffic(args):
    """HBM bytes per step_kernel launch from the committed PMC passes (profiles/traffic_r02_step.json), if
    they were taken on this workload."""
    path = os.path.join(ROOT, "profiles", "traffic_r02_step.json")
    try:
        with open(path) as f:
            tj = json.load(f)
        if tj.get("workload") == f"step_{args.method}_{args.patients}x{args.T}":
            return tj.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def fused_run(args, dev, coh, arm_cf, coh2=None, arm_cf2=None):
    """Time the fused step (insite_fit_rollout_f64: step_kernel) on the C2 cohort.  One launch per step runs
    the discovery of step i (gram + in-launch reduction + the F = 7 STLSQ in its last block) and, on the
    other blocks of the same resident round, the rollout of step i-1 with the coefficients discovery i-1
    wrote (two coefficient buffers, ping-pong).  K timed launches = K discoveries + K rollouts.
    With a second cohort (coh2, the default: --no-rotate turns it off) the steps alternate between the two:
    step i discovers cohort i % 2 and rolls cohort (i - 1) % 2 out into that cohort's own y, so consecutive
    reads of one cohort's x are 480 MB of other traffic apart -- more than the 256 MB Infinity Cache, whose
    hits the PMC byte counters count (MI355X_MICROARCH.md) -- and no step re-reads resident data."""
    from insite_amd import ops
    N, T = args.patients, args.T
    lib = coh.lib
    F = lib.n_terms
    f64 = torch.float64
    cohs = [coh, coh2 if coh2 is not None else coh]
    arms = [arm_cf, arm_cf2 if coh2 is not None else arm_cf]
    coefs = [torch.zeros((2, F), dtype=f64, device=dev) for _ in range(2)]
    masks = [torch.zeros((2, F), dtype=torch.int8, device=dev) for _ in range(2)]
    iters = [torch.zeros((2,), dtype=torch.int32, device=dev) for _ in range(2)]
    Gs = [torch.zeros((2, F, F), dtype=f64, device=dev) for _ in range(2)]
    bs = [torch.zeros((2, F), dtype=f64, device=dev) for _ in range(2)]
    y1 = torch.empty((T, N), dtype=f64, device=dev)
    ys = [y1, torch.empty((T, N), dtype=f64, device=dev) if coh2 is not None else y1]
    y = ys[0]
    # step -1: a plain discovery of the cohort step 0 rolls out gives the first rollout its model
    c1 = cohs[1]
    ops.sindy_fit(c1.x, c1.u, c1.arm, c1.rows, c1.dt, lib, 0.1, 0.5, out=(coefs[1], masks[1], iters[1], Gs[1],
                                                                          bs[1]), layout="time")
    # plan j: discovery of cohort j into coefs[j] | rollout of cohort 1 - j with coefs[1 - j] into its y
    plans = [ops.plan_fit_rollout(cohs[j].x, cohs[j].u, cohs[j].arm, cohs[j].rows, cohs[j].dt, lib, 0.1, 0.5,
                                  cohs[1 - j].y0, cohs[1 - j].u, arms[1 - j], coefs[1 - j], cohs[1 - j].dt,
                                  method=args.method, T=T, y_out=ys[1 - j],
                                  out=(coefs[j], masks[j], iters[j], Gs[j], bs[j]), gram_blocks=args.gram_blocks)
             for j in range(2)]
    st = torch.cuda.current_stream(dev)
    fast = [p.bind(st) for p in plans]
    if args.fused_graph:    # the ping-pong pair of launches captured once in a HIP graph, replayed
        for p in plans:
            p()
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            gs = torch.cuda.current_stream(dev)
            plans[0](gs)
            plans[1](gs)
        pair = graph.replay
        fast = [pair, lambda: None]     # step 2i replays the pair (steps 2i, 2i+1); step 2i+1 is already in it
    def run_steps(n):                   # n steps = n launches (graph: n // 2 pair replays + an odd last one)
        for i in range(n - (n % 2 if args.fused_graph else 0)):
            fast[i % 2]()
        if args.fused_graph and n % 2:
            plans[0](st)

    run_steps(args.warmup)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(args.steps)
    host_ms = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize(dev)
    ms_step = (time.perf_counter() - t0) / args.steps * 1e3
    last = (args.steps - 1) % 2
    # instrumented pass: HIP timing events on the launch stream around batches of KB back-to-back launches
    # (an event record costs ~20 us of queue time on ROCm 7.2, so never one per launch), divided by KB
    hip = HipEvents()
    # batches of >= 100 launches: an event record puts ~20 us of dead queue time into the stream (ROCm 7.2,
    # profiles/r02/c2_pipeline_trace.txt), which over round 5's 20-launch batches read as ~1 us more per launch than
    # the timed region's own wall clock (What's weak 4)
    KB, NBAT = max(args.steps, 100), 3
    tevs = [(hip.create(timing=True), hip.create(timing=True)) for _ in range(NBAT)]
    for e0, e1 in tevs:
        hip.record(e0, st.cuda_stream)
        run_steps(KB)
        hip.record(e1, st.cuda_stream)
    torch.cuda.synchronize(dev)
    step_ms = float(np.mean([hip.elapsed_ms(e0, e1) for e0, e1 in tevs])) / KB
    rb, gb = rollout_bytes(N, T, arm_bits=1), gram_bytes(N, T)
    return {"ms_step": ms_step, "host_ms": host_ms, "step_ms": step_ms, "KB": KB, "NBAT": NBAT,
            "coef": coefs[last], "mask": masks[last], "y": ys[last], "rb": rb, "gb": gb, "rotated": coh2 is not None,
            "frac": (rb + gb) / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}


def deferred_run(args, dev, coh, arm_cf, coh2=None, arm_cf2=None):
    """Time the deferred fused step (insite_fit_rollout_deferred_f64: step_deferred_kernel).  One launch per
    step: the gram streaming of a cohort into a partial slot, the finalisation (reduction + STLSQ) of the
    previous launch's cohort by one block, and the rollout of a cohort with coefficients finalised one launch
    earlier still (three coefficient buffers); nothing in a launch waits on anything else in it.
    --dstreams S (default 1): S independent deferred streams of cohorts, launch k on stream k % S, each with
    its own workspace, slots and buffers -- a launch depends only on the previous launch of its own stream, so
    the next stream's launch fills the CU slots the current one's last waves leave idle (the end of every
    launch is a 48-73 us spread of wave finish times, profiles/r03/v16_timing_deferred.jsonl).  Two cohorts
    per stream alternate (one per stream with --no-rotate), so no launch re-reads x that is still resident."""
    from insite_amd import ops, cohort
    N, T = args.patients, args.T
    lib = coh.lib
    F = lib.n_terms
    f64 = torch.float64
    S = max(1, args.dstreams)
    pool = [(coh, arm_cf)] + ([(coh2, arm_cf2)] if coh2 is not None else [])
    need = 2 * S if coh2 is not None else S
    while len(pool) < need:   # more cohorts for the extra streams (distinct seeds)
        sd = args.seed * 1000 + 700 + len(pool)
        c = cohort.synthetic_pkpd(N, T, seed=sd, device=dev, equation="EQ_4_C", layout="time")
        pool.append((c, cohort.counterfactual_arms(c.arm, T, seed=sd, layout=bits_layout(args.arm_format))))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    lanes = []   # per stream: (its cohorts, outs ring, ys, workspace)
    for si in range(S):
        mine = pool[si::S]
        outs = [(torch.zeros((2, F), dtype=f64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
                 torch.zeros((2,), dtype=torch.int32, device=dev), torch.zeros((2, F, F), dtype=f64, device=dev),
                 torch.zeros((2, F), dtype=f64, device=dev)) for _ in range(3)]
        ys = [torch.empty((T, N), dtype=f64, device=dev) for _ in mine]
        # the stream's steps 0 and 1 roll out with coefficients from before the stream: plain discoveries
        for j in (1, 2):
            c = mine[(j - 1) % len(mine)][0]
            ops.sindy_fit(c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, out=outs[j], layout="time")
        lanes.append((mine, outs, ys, ops.Workspace()))
    torch.cuda.synchronize(dev)

    def plan(si, k, finalize):   # stream si's step k: gram of its cohort k % m -> slot k % 2; finalise the
        mine, outs, ys, ws = lanes[si]   # previous step's cohort -> outs[(k-1) % 3]; roll cohort k % m out
        m = len(mine)
        c, a = mine[k % m]
        return ops.plan_fit_rollout_deferred(c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, c.y0, c.u, a,
                                             outs[(k - 2) % 3][0], c.dt, k % 2, finalize, ws, method=args.method,
                                             T=T, y_out=ys[k % m], out=outs[(k - 1) % 3],
                                             gram_blocks=args.gram_blocks)
    for si in range(S):          # each stream's first call has nothing to finalise
        plan(si, 0, False)(streams[si])
    fast = [[plan(si, k, True).bind(streams[si]) for k in range(6)] for si in range(S)]  # cycle: slot k%2, bufs k%3
    pos = [1] * S
    turn = [0]

    def run_steps(n):            # step i on stream i % S
        for _ in range(n):
            si = turn[0] % S
            fast[si][pos[si] % 6]()
            pos[si] += 1
            turn[0] += 1

    run_steps(args.warmup)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(args.steps)
    host_ms = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize(dev)
    ms_step = (time.perf_counter() - t0) / args.steps * 1e3
    # instrumented pass: timing events on stream 0 around batches of KB steps; the other streams' last launches
    # are joined into stream 0 before the closing event (one ordering event per stream per batch)
    hip = HipEvents()
    # batches of >= 100 launches (>= 10 for launches over 0.5 ms): each event record is ~20 us of dead queue time
    # (ROCm 7.2), ~1 us a launch over round 5's 20-launch batches (What's weak 4)
    KB, NBAT = max(args.steps, 100 if args.patients * args.T <= 50_000_000 else 10), 3
    tevs = [(hip.create(timing=True), hip.create(timing=True)) for _ in range(NBAT)]
    joins = [hip.create() for _ in range(S)]
    st0 = streams[0].cuda_stream
    for e0, e1 in tevs:
        torch.cuda.synchronize(dev)
        hip.record(e0, st0)
        for si in range(1, S):
            hip.wait(streams[si].cuda_stream, e0)
        run_steps(KB)
        for si in range(1, S):
            hip.record(joins[si], streams[si].cuda_stream)
            hip.wait(st0, joins[si])
        hip.record(e1, st0)
    torch.cuda.synchronize(dev)
    step_ms = float(np.mean([hip.elapsed_ms(e0, e1) for e0, e1 in tevs])) / KB
    rb, gb = rollout_bytes(N, T, arm_bits=1), gram_bytes(N, T)
    mine, outs, ys, _ = lanes[(turn[0] - 1) % S]
    last = pos[(turn[0] - 1) % S] - 1
    fin = outs[(last - 1) % 3]
    # the last launch rolled cohort mine[last % m] out with the model finalised one launch earlier -- that of the
    # same data cohort two launches back (m = 2): the bench line's parity check compares THAT model and y
    used = outs[(last - 2) % 3]
    return {"ms_step": ms_step, "host_ms": host_ms, "step_ms": step_ms, "KB": KB, "NBAT": NBAT,
            "coef": fin[0], "mask": fin[1], "y": ys[last % len(mine)], "rb": rb, "gb": gb, "rotated": coh2 is not None,
            "streams": S, "frac": (rb + gb) / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "roll_coef": used[0], "roll_mask": used[1], "roll_cohort": mine[last % len(mine)]}


def c2_parity(dev, coh, arm_bits, coef, mask, y, n_sample=4096, seed=11, pooled=False):
    """The metric's "RMSE vs CPU ref" for the benched cohort (after the timed region): the oracle
    (oracle/insite_ref.py: the reference's SINDy.fit + RK4 scan restated, sindy.py:190-192, 371-431) fits the SAME
    cohort whose rollout the last timed launch wrote (C2: 100k x 200; the north-star step: 1M x 500), and rolls a
    sample of its rows out with its own model; the line reports support equality, coefficient L-inf (GPU vs oracle
    model) and the trajectory RMSE / max relative error of the GPU y on the sampled rows against the oracle's.
    ``pooled``: the whole-cohort Gram in patient chunks and the sampled rollouts on a spawned pool of the host's
    workers (the chunk Grams summed in chunk order; the 1M x 500 cohort is 500M samples)."""
    sys.path.insert(0, ROOT)
    from oracle import insite_ref as R
    N, T = coh.arm.numel(), coh.x.size(0)
    exps = coh.lib.exps.astype(np.int64)
    u, arm = coh.u.cpu().numpy(), coh.arm.cpu().numpy().astype(np.int64)
    rows = coh.rows.cpu().numpy()
    if not np.all(rows == rows[0]):
        return {"skipped": "ragged rows (the vectorised oracle Gram needs equal rows)"}
    t0 = time.perf_counter()
    W = host_info()["workers"] if pooled else 1
    if pooled:
        bounds = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(N), 2 * W) if c.size]
        gb = parity_map(_par_gram_job, [(coh.x[:, lo:hi].t().contiguous().cpu().numpy(), u[lo:hi], arm[lo:hi],
                                         int(rows[0]), coh.dt, exps) for lo, hi in bounds])
        G, b = sum(q[0] for q in gb), sum(q[1] for q in gb)
    else:
        x = coh.x[:, :N].t().contiguous().cpu().numpy()
        G, b = R.gram_moments_vectorized(x, u, arm, int(rows[0]), coh.dt, exps)
    cr = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    cg, mg = coef.cpu().numpy(), mask.cpu().numpy()
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([rng.choice(N, min(n_sample, N), replace=False), np.arange(min(64, N)),
                                    np.arange(max(0, N - 64), N)]))
    it = torch.as_tensor(idx, device=dev)
    arms = _unpack_bits_rows(arm_bits, it, arm_bits.size(0) if arm_bits.dim() == 2 else arm_bits.size(1))
    y0s, us = coh.y0[it].cpu().numpy(), coh.u[it].cpu().numpy()
    if pooled:
        parts = [c for c in np.array_split(np.arange(idx.size), 4 * W) if c.size]
        ref = np.concatenate(parity_map(_par_roll_job, [(y0s[c], us[c], arms[c, :y.size(0)], cr, exps, coh.dt, "rk4")
                                                        for c in parts]))
    else:
        ref = R.rollout(y0s, us, arms[:, :y.size(0)], cr, exps, coh.dt, method="rk4")
    el = time.perf_counter() - t0
    got = y.index_select(1, it).t().cpu().numpy()
    d = got - ref
    return {"oracle": "oracle/insite_ref.py (numpy restatement; gram_moments_vectorized + stlsq_gram + rollout rk4)",
            "cohort": f"the last timed launch's rollout cohort ({N} x {T}, the model it used)",
            "support_equal": bool(np.array_equal(mg != 0, cr != 0)),
            "coef_linf": float(np.max(np.abs(cg - cr))),
            "y_rmse": float(np.sqrt(np.mean(d ** 2))),
            "y_max_rel": float(np.max(np.abs(d) / np.maximum(np.abs(ref), 1e-300))),
            "rows_sampled": int(idx.size), "steps_per_row": int(y.size(0)), "oracle_seconds": el,
            **({"oracle_workers": W} if pooled else {}),
            "tolerances": {"coef_linf": 1e-8, "y_rmse": 1e-6}}


def c2_fused(args, dev, coh, arm_cf, cpu):
    """C2 at N = 1 with one step_kernel launch per step (--mode fused); see fused_run.  Two cohorts rotate
    (a second seed) unless --no-rotate."""
    from insite_amd import ops, cohort
    N, T = args.patients, args.T
    lib = coh.lib
    F = lib.n_terms
    coh2 = arm_cf2 = None
    if not args.no_rotate:
        coh2 = cohort.synthetic_pkpd(N, T, seed=args.seed * 1000 + 500, device=dev, equation="EQ_4_C", layout="time")
        arm_cf2 = cohort.counterfactual_arms(coh2.arm, T, seed=args.seed * 1000 + 500,
                                             layout=bits_layout(args.arm_format))
    deferred = args.mode == "deferred"
    fr = (deferred_run if deferred else fused_run)(args, dev, coh, arm_cf, coh2, arm_cf2)
    ms_step, host_ms, step_ms, KB, NBAT = fr["ms_step"], fr["host_ms"], fr["step_ms"], fr["KB"], fr["NBAT"]
    y = fr["y"]
    st = torch.cuda.current_stream(dev)

    iso = None
    if args.isolated:   # the two halves as separate launches, back to back on one stream
        def timed(fn, n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(n):
                fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / n
        # with rotation on, the isolated launches alternate between the two cohorts (and their y) as well
        cs = [(coh, arm_cf), (coh2, arm_cf2)] if coh2 is not None else [(coh, arm_cf)]
        y2 = torch.empty_like(y) if coh2 is not None else y
        gps = [ops.plan_sindy_fit(c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, layout="time").bind(st) for c, _ in cs]
        rps = [ops.plan_rollout(c.y0, c.u, a, fr["coef"], lib, c.dt, method=args.method, T=T, out=yy,
                                layout="time_bits").bind(st) for (c, a), yy in zip(cs, (y, y2))]
        gi, ri = iter(range(10 ** 9)), iter(range(10 ** 9))
        iso = {"discovery_avg_launch_ms": timed(lambda: gps[next(gi) % len(gps)](), 20),
               "rollout_avg_launch_ms": timed(lambda: rps[next(ri) % len(rps)](), 20),
               "rotated": coh2 is not None}

    sup = fr["mask"].cpu().numpy()
    ok = bool(torch.isfinite(y).all().item())
    rb, gb = fr["rb"], fr["gb"]
    achieved = (rb + gb) / (step_ms * 1e-3) / 1e9
    out = {
        "metric": METRIC,
        "value": N / (ms_step * 1e-3),
        "unit": "patient-trajectories/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: on-device EQ_4_C PK/PD cohort (reference distributions, Euler-5 truth + 0.01 noise)",
        "config": {
            "workload": f"C2: PK/PD {N // 1000}k patients/GPU x {T} steps fp64 - discovery (savgol+FD4+poly2 "
                        f"library+Gram, STLSQ) + {args.method.upper()} counterfactual rollout",
            "patients_per_gpu": N, "T": T, "rows_per_patient": T - 2, "library_terms": F,
            "parallelism": "patient-shard x1", "mode": args.mode, "gram_blocks": args.gram_blocks or "default",
            "discovered_support": sup.tolist(), "finite": ok,
            "cohorts_rotated": (2 if fr["rotated"] else 1) * fr.get("streams", 1),
            **({"deferred_streams": fr["streams"]} if deferred else {}),
        },
        "host_submit_ms_per_step": host_ms,
        "roofline": {
            "kernel": (f"step_deferred_kernel (gram streaming | finalisation of the previous step's gram: reduction + "
                       f"STLSQ | {args.method} bit-arm rollout)") if deferred else
                      f"step_kernel (discovery: gram + in-launch reduction + STLSQ | {args.method} bit-arm rollout)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": None,
            "algorithmic_bytes_per_launch": rb + gb,
            "algorithmic_bytes_split": {"discovery_x_read": gb, "rollout_y_written": rb},
            "avg_launch_ms": step_ms,
            "avg_ms_source": f"HIP timing events on the launch stream around {NBAT} batches of {KB} back-to-back "
                             f"{'step_deferred_kernel' if deferred else 'step_kernel'} launches, divided by the batch "
                             "size (one launch = one step)",
            "layout": "time-major x[T,N] read, 1-bit arm mask [T,N/32], y[T,N] written",
        },
        "timed_region": ("one step_deferred_kernel launch per step on one stream: gram of cohort i | finalisation "
                         "(block reduction + STLSQ) of cohort i-1 | rollout with the coefficients of cohort i-2 (three "
                         "coefficient buffers); no events or cross-stream waits inside the timed region") if deferred
                        else "one step_kernel launch per step on one stream: discovery of step i | rollout of step "
                             "i-1 (two coefficient buffers); no events or cross-stream waits inside the timed region",
        "step_aggregate": {"algorithmic_bytes": rb + gb, "achieved_GBps": (rb + gb) / (ms_step * 1e-3) / 1e9,
                           "frac": (rb + gb) / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS},
        "pipeline_alternative": "bench.py --mode pipeline: gram | rollout on two streams (the N > 1 schedule); "
                                "within a few % of this line, ahead over long runs (profiles/r02/fused_sweep/)",
    }
    t3 = (traffic_for("c2", "step_deferred_kernel" if deferred else "step_kernel")
          if fr["rotated"] and args.patients == 100_000 and args.T == 200 else None)
    out["roofline"]["traffic"] = t3 if (t3 is not None or deferred) else step_traffic(args)
    if iso is not None:
        out["isolated"] = dict(iso, discovery_frac=gb / (iso["discovery_avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                               rollout_frac=rb / (iso["rollout_avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS)
    if "roll_coef" in fr and not args.no_parity:
        rc_, ra_ = fr["roll_cohort"]
        out["parity"] = c2_parity(dev, rc_, ra_, fr["roll_coef"], fr["roll_mask"], y)
    if not args.no_north_star:
        del y
        torch.cuda.empty_cache()
        out["north_star_rollout"] = north_star_rollout(args, dev, fr["coef"], lib)
    # the two larger configurations in the driver's own line: BASELINE.json north_star's
    # 1M x 500 through the headline kernel, and C3 (configs[2], the largest single-GPU configuration), each with its
    # roofline and oracle parity; the C2 figures above are the line's value.  A failure here never costs the line.
    fr = None
    torch.cuda.empty_cache()
    if not args.no_north_star and deferred and args.patients == 100_000 and args.T == 200:
        try:
            out["north_star_step"] = north_star_step(args, dev)
        except Exception as exc:
            out["north_star_step"] = {"error": f"{type(exc).__name__}: {exc}"}
        torch.cuda.empty_cache()
    if not args.no_c3_block and deferred and args.patients == 100_000 and args.T == 200:
        try:
            c3 = c3_measure(args, dev, 1_000_000, 500, 5, 2, not args.no_parity)
            out["c3"] = {k: c3[k] for k in ("value", "ms_per_step", "steps", "warmup", "dtype", "config", "roofline",
                                            "rollout", "parity") if k in c3}
            out["c3"]["note"] = ("BASELINE configs[2] (5-state + binary treatment, 1M x 500): discovery (S-state Gram "
                                 "on f64 MFMA + STLSQ per state) + RK4 rollout; CPU leg and PMC traffic in the "
                                 "standalone line (bench.py --config c3)")
        except Exception as exc:
            out["c3"] = {"error": f"{type(exc).__name__}: {exc}"}
        torch.cuda.empty_cache()
    if cpu is not None:
        out["cpu_baseline"] = cpu
    emit(out)


def c2_lagged(args, dev, world, rank, coh, arm_cf, cpu, collective):
    """C2 at N GPUs (the default at N > 1; ``--mode lagged`` also at N = 1, with --force-collective to put the
    single-rank RCCL all-reduce in): ONE insite_fit_rollout_lagged_f64 launch per step -- the step_deferred_kernel
    timed at N = 1 with its finalisation split into a reduction role (rank-local G|b) and a solve role (an
    all-reduced G|b) -- and one RCCL all-reduce of a K-fit bucket per K launches (insite_amd.dist.LaggedSchedule):
    by default (--lag-delay 1, --lag-k 16) issued async and waited for by the launch stream only K launches later,
    so the collective runs beside the launches (delay 0: in order on the launch stream).  Two cohorts per rank rotate, as at N = 1, so no launch
    re-reads x still resident in the 256 MB Infinity Cache.  value = all ranks' patients / the max-over-ranks
    step time (weak scaling: 100k patients per GPU)."""
    from insite_amd import ops, cohort
    from insite_amd import dist as idist
    N, T = args.patients, args.T
    lib = coh.lib
    F = lib.n_terms
    f64 = torch.float64
    K = max(1, args.lag_k)
    sched = idist.LaggedSchedule(K, delay=args.lag_delay)
    sd = args.seed * 1000 + 500 + rank
    coh2 = cohort.synthetic_pkpd(N, T, seed=sd, device=dev, equation="EQ_4_C", layout="time")
    cohs = [(coh, arm_cf), (coh2, cohort.counterfactual_arms(coh2.arm, T, seed=sd, layout=bits_layout(args.arm_format)))]
    buckets = [idist.MomentBucket(K, 2, F, dev) for _ in range(sched.NB)]
    ring = [(torch.zeros((2, F), dtype=f64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
             torch.zeros((2,), dtype=torch.int32, device=dev)) for _ in range(3)]
    ys = [torch.empty((T, N), dtype=f64, device=dev) for _ in range(2)]
    scratch = (torch.zeros((2, F, F), dtype=f64, device=dev), torch.zeros((2, F), dtype=f64, device=dev))
    ws = ops.Workspace()
    # the prologue's rollouts (launches < K + 2 have no solved model yet) use a plain fit of each cohort
    warm = [ops.sindy_fit(c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, layout="time")[0] for c, _ in cohs]
    st = torch.cuda.current_stream(dev)

    def plan(k):
        p = sched.launch(k)
        c, _ = cohs[k % 2]
        red = buckets[p["reduce"][1]].bufs[p["reduce"][2]] if p["reduce"] else None
        fit_in = fit_out = None
        if p["fit"]:
            _, bi, pos, r = p["fit"]
            fit_in, fit_out = (buckets[bi].bufs[pos].G, buckets[bi].bufs[pos].b), ring[r]
        if p["rollout"]:
            rc_, r = p["rollout"]
            (rcoh, rbits), cin, yy = cohs[rc_ % 2], ring[r][0], ys[rc_ % 2]
        else:
            (rcoh, rbits), cin, yy = cohs[k % 2], warm[k % 2], ys[k % 2]
        launch = ops.plan_fit_rollout_lagged(
            c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, rcoh.y0, rcoh.u, rbits, cin, rcoh.dt, p["slot"],
            p["reduce"] is not None, ws, (red.G, red.b) if red is not None else scratch, fit_in=fit_in,
            fit_out=fit_out, method=args.method, T=T, y_out=yy, gram_blocks=args.gram_blocks).bind(st)
        ar = p["allreduce_after"]
        return launch, ar, p

    P = sched.period_of()
    k0 = sched.lag                               # the first steady-state launch
    steady = {}
    for k in range(k0, k0 + P):
        steady[k % P] = plan(k)
    pending = {}                                 # delay 1: bucket -> the in-flight all-reduce's work handle

    def one(k):
        launch, ar, p = plan(k) if k < k0 else steady[k % P]
        if p["wait_before"] is not None and p["wait_before"] in pending:
            pending.pop(p["wait_before"]).wait()     # the launch stream waits for the collective (no host block)
        launch()
        if ar is not None and collective:        # the only collective: one per K launches
            if sched.D:
                h = idist.reduce_bucket(buckets[ar], force=args.force_collective, async_op=True)
                if h is not None:
                    pending[ar] = h
            else:                                # in order on the launch stream
                idist.reduce_bucket(buckets[ar], force=args.force_collective)

    kk = [0]

    def run_steps(n):
        for _ in range(n):
            one(kk[0])
            kk[0] += 1

    run_steps(k0 + args.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(args.steps)
    host_ms = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = idist.max_over_ranks(time.perf_counter() - t0, dev)
    ms_step = el / args.steps * 1e3
    last = kk[0] - 1
    # instrumented pass: HIP events around batches of KB launches (+ their collectives), divided by KB
    hip = HipEvents()
    KB, NBAT = max(args.steps // K * K, 2 * K), 3
    tevs = [(hip.create(timing=True), hip.create(timing=True)) for _ in range(NBAT)]
    for e0, e1 in tevs:
        hip.record(e0, st.cuda_stream)
        run_steps(KB)
        hip.record(e1, st.cuda_stream)
    torch.cuda.synchronize(dev)
    step_ms = float(np.mean([hip.elapsed_ms(e0, e1) for e0, e1 in tevs])) / KB
    last = kk[0] - 1
    p_last = sched.launch(last)
    rc_, r = p_last["rollout"]
    coef_used, mask_used = ring[r][0], ring[r][1]
    y = ys[rc_ % 2]
    rb, gb = rollout_bytes(N, T, arm_bits=1), gram_bytes(N, T)
    out = None
    if rank == 0:
        achieved = (rb + gb) / (step_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": N * world / (ms_step * 1e-3),
            "unit": "patient-trajectories/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: on-device EQ_4_C PK/PD cohorts (reference distributions, Euler-5 truth + 0.01 noise)",
            "config": {
                "workload": f"C2: PK/PD {N // 1000}k patients/GPU x {T} steps fp64 - discovery (savgol+FD4+poly2 "
                            f"library+Gram, one RCCL all-reduce per {K} fits, STLSQ) + {args.method.upper()} "
                            "counterfactual rollout",
                "patients_per_gpu": N, "T": T, "rows_per_patient": T - 2, "library_terms": F,
                "parallelism": f"patient-shard x{world}" + (" (single-rank RCCL group: --force-collective)"
                                                             if args.force_collective and world == 1 else ""),
                "mode": "lagged", "fits_per_allreduce": K, "lag_launches": sched.lag,
                "allreduce": ("async, waited K launches later (LaggedSchedule delay 1)" if sched.D else
                              "in order on the launch stream"),
                "discovered_support": mask_used.cpu().numpy().tolist(),
                "finite": bool(torch.isfinite(y).all().item()), "cohorts_rotated_per_rank": 2,
            },
            "host_submit_ms_per_step": host_ms,
            "roofline": {
                "kernel": "step_deferred_kernel, lagged (gram streaming | reduction of the previous slot to rank-local "
                          "G|b | STLSQ of an all-reduced G|b | rk4 bit-arm rollout)",
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                "algorithmic_bytes_per_launch": rb + gb,
                "algorithmic_bytes_split": {"discovery_x_read": gb, "rollout_y_written": rb},
                "avg_launch_ms": step_ms,
                "avg_ms_source": f"HIP timing events on the launch stream around {NBAT} batches of {KB} launches "
                                 f"(with their {KB // K} bucket all-reduces), divided by the batch size",
            },
            "timed_region": f"one lagged launch per step on one stream + one all-reduce of a {K}-fit G|b bucket "
                            "per K launches (" + ("issued async on RCCL's stream, the launch stream waiting for it K "
                                                  "launches later" if sched.D else "on the same stream, in order") + ")",
        }
        if cpu is not None:
            out["cpu_baseline"] = cpu
    return out, (cohs[rc_ % 2], coef_used, mask_used, y)


def north_star_step(args, dev):
    """BASELINE.json north_star's own configuration through the headline kernel: the full deferred
    step -- step_deferred_kernel: gram streaming of cohort k | finalisation (reduction + STLSQ) of cohort k-1 | RK4
    bit-arm rollout of cohort k-2 with its own model -- on 1M patients x 500 steps fp64, two rotating EQ_4_C cohorts
    (2 x 4 GB of x, 2 x 4 GB of y: no launch re-reads data the Infinity Cache holds), ``--ns-steps`` timed launches,
    the roofline from HIP events on the launch stream, and the oracle parity of the model and the trajectories the
    last timed launch used (the whole-cohort oracle fit on the host's workers)."""
    from insite_amd import cohort
    ns = argparse.Namespace(**vars(args))
    ns.patients, ns.T, ns.steps, ns.warmup, ns.dstreams, ns.gram_blocks = 1_000_000, 500, max(2, args.ns_steps), 3, 1, 0
    N, T = ns.patients, ns.T
    sd = [args.seed * 1000 + 900, args.seed * 1000 + 901]
    cohs = [cohort.synthetic_pkpd(N, T, seed=s_, device=dev, equation="EQ_4_C", layout="time") for s_ in sd]
    arms = [cohort.counterfactual_arms(c.arm, T, seed=s_, layout=bits_layout(args.ns_arms)) for c, s_ in zip(cohs, sd)]
    torch.cuda.synchronize(dev)
    fr = deferred_run(ns, dev, cohs[0], arms[0], cohs[1], arms[1])
    rb, gb = fr["rb"], fr["gb"]
    out = {"workload": "north star: PK/PD EQ_4_C 1M patients x 500 steps fp64 - discovery (savgol+FD4+poly2 "
                       "library+Gram, STLSQ) + RK4 counterfactual rollout, one step_deferred_kernel launch per step",
           "patients": N, "T": T, "steps": ns.steps, "warmup": ns.warmup, "cohorts_rotated": 2,
           "ms_per_step": fr["ms_step"], "patient_trajectories_per_s": N / (fr["ms_step"] * 1e-3),
           "discovered_support": fr["mask"].cpu().numpy().tolist(),
           "finite": bool(torch.isfinite(fr["y"]).all().item()),
           "roofline": {"kernel": "step_deferred_kernel<true, rk4>", "bound": "hbm", "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "achieved": (rb + gb) / (fr["step_ms"] * 1e-3) / 1e9,
                        "frac": (rb + gb) / (fr["step_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                        "avg_launch_ms": fr["step_ms"], "algorithmic_bytes_per_launch": rb + gb,
                        "algorithmic_bytes_split": {"discovery_x_read": gb, "rollout_y_written": rb},
                        "avg_ms_source": f"HIP timing events on the launch stream around {fr['NBAT']} batches of "
                                         f"{fr['KB']} back-to-back launches, divided by the batch size",
                        "traffic": traffic_for("ns", "step_deferred_kernel", args=args)},
           "step_aggregate_frac": (rb + gb) / (fr["ms_step"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
           "target": "north_star: >= 0.40 of the HBM roofline at 1M x 500 on one GPU"}
    if not args.no_parity:
        rc_, ra_ = fr["roll_cohort"]
        out["parity"] = c2_parity(dev, rc_, ra_, fr["roll_coef"], fr["roll_mask"], fr["y"], pooled=True)
    return out


def ns_main(args):
    """--config ns: the north_star_step block of the default line as a line of its own (counter / profiler runs)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ns = north_star_step(args, dev)
    emit({"metric": METRIC, "value": ns["patient_trajectories_per_s"], "unit": "patient-trajectories/s", "n_gpus": 1,
          "steps": ns["steps"], "warmup": ns["warmup"], "ms_per_step": ns["ms_per_step"], "higher_is_better": True,
          "scaling": "weak", "vs_baseline": None, "dtype": "f64",
          "data": "synthetic: on-device EQ_4_C PK/PD cohorts (reference distributions, Euler-5 truth + 0.01 noise)",
          "config": {"workload": ns["workload"], "patients": ns["patients"], "T": ns["T"]},
          **{k: v for k, v in ns.items() if k in ("roofline", "parity", "discovered_support", "finite",
                                                  "step_aggregate_frac")}})


def north_star_rollout(args, dev, coef, lib):
    """The 1M x 500 RK4 rollout alone (the north star's >= 40 % roofline target), events around each launch."""
    from insite_amd import ops
    Nn, Tn = 1_000_000, 500
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    y0n = torch.rand(Nn, generator=g, device=dev, dtype=torch.float64) * 49 + 1
    un = torch.rand((Nn, 2), generator=g, device=dev, dtype=torch.float64) * 0.1 + 0.45
    flip = torch.randint(0, Tn, (Nn, 1), generator=g, device=dev)
    armn = torch.zeros((Tn, Nn), dtype=torch.int8, device=dev)
    armn[:] = (torch.arange(Tn, device=dev)[:, None] >= flip[:, 0][None, :]).to(torch.int8)
    nlay = "time_bits" if args.arm_format in ("bits", "tiles") else "time"
    if nlay == "time_bits":
        armn = ops.pack_arm_bits(armn, Nn)
        if args.ns_arms == "tiles":     # the tile-major bits (one 256-B run per tile and 32-step group)
            armn = ops.tile_major_bits(armn, Nn)
    yn = torch.empty((Tn, Nn), dtype=torch.float64, device=dev)
    for _ in range(3):
        ops.rollout(y0n, un, armn, coef, lib, 10.0 / Tn, method="rk4", out=yn, layout=nlay)
    evs = []
    for _ in range(10):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream(dev))
        ops.rollout(y0n, un, armn, coef, lib, 10.0 / Tn, method="rk4", out=yn, layout=nlay)
        e1.record(torch.cuda.current_stream(dev))
        evs.append((e0, e1))
    torch.cuda.synchronize(dev)
    ms = float(np.mean([a.elapsed_time(b_) for a, b_ in evs]))
    bn = rollout_bytes(Nn, Tn, arm_bits=1 if nlay == "time_bits" else 8)
    return {"patients": Nn, "T": Tn, "method": "rk4",
            "layout": nlay + (" (tile-major bits)" if nlay == "time_bits" and args.ns_arms == "tiles" else ""),
            "avg_launch_ms": ms,
            "algorithmic_bytes": bn, "achieved_GBps": bn / (ms * 1e-3) / 1e9,
            "frac_of_8TBps": bn / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "patient_trajectories_per_s": Nn / (ms * 1e-3)}


_JSON_OUT = None


def quiet_stdout():
    """Keep the bench's stdout to its ONE JSON line: libraries that print banners on fd 1 (RCCL's "RCCL version"
    block at communicator init, tqdm, ...) are sent to stderr from here on; ``emit`` writes to the saved fd."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit(obj):
    print(json.dumps(obj), file=_JSON_OUT or sys.stdout, flush=True)


def main():
    args = parse()
    launch_ranks(args)   # (N > 1 without torchrun: re-launches through torchrun as a child and exits here)
    quiet_stdout()
    if args.config == "f4":
        return f4_main(args)
    if args.config == "c4":
        return c4_main(args)
    if args.config == "insite4":
        return insite4_main(args)
    if args.config == "insite":
        return insite_main(args)
    if args.config == "c3":
        return c3_main(args)
    if args.config == "c5":
        return c5_main(args)
    if args.config == "ns":
        return ns_main(args)
    # the CPU leg runs first, while this process has no GPU context (its worker pool forks)
    cpu = None
    if os.environ.get("WORLD_SIZE", "1") == "1" and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample, args.T, args.method, args.seed)
    world, rank, dev = dist_setup(force_group=args.force_collective)
    if args.force_collective and args.mode not in ("pipeline", "lagged"):
        args.mode = "lagged"
    collective = world > 1 or args.force_collective   # the N > 1 data path all-reduces G|b

    from insite_amd import ops, cohort
    from insite_amd import dist as idist

    N, T = args.patients, args.T
    coh = cohort.synthetic_pkpd(N, T, seed=args.seed * 1000 + rank, device=dev, equation="EQ_4_C",
                                layout=args.layout)
    # time-major arm sequences / trajectories: one contiguous run per step ("HBM layout")
    roll_layout = (bits_layout(args.arm_format) if args.arm_format != "int8" else "time") if args.layout == "time" \
        else args.layout
    arm_cf = cohort.counterfactual_arms(coh.arm, T, seed=args.seed * 1000 + rank, layout=roll_layout)
    lib = coh.lib
    F = lib.n_terms
    y0 = coh.y0
    if args.mode is None:   # N = 1: one deferred fused launch per step; N > 1: the same kernel, lagged
        args.mode = "deferred" if world == 1 and not args.force_collective else "lagged"
    if args.mode in ("fused", "deferred") and world > 1:
        raise SystemExit(f"--mode {args.mode} is single-GPU (the all-reduce sits between the gram and STLSQ): "
                         "use --mode lagged (the default at N > 1) or pipeline")
    if args.mode in ("fused", "deferred"):
        return c2_fused(args, dev, coh, arm_cf, cpu)
    if args.mode == "lagged":
        out, (rcoh, rcoef, rmask, ry) = c2_lagged(args, dev, world, rank, coh, arm_cf, cpu, collective)
        if out is not None:
            if not args.no_parity:
                out["parity"] = c2_parity(dev, rcoh[0], rcoh[1], rcoef, rmask, ry) if world == 1 else {
                    "skipped": "N > 1: each rank's model is the all-rank fit; the single-rank parity is tests/"
                               "test_gpu_deferred.py and test_dist.py::test_lagged_schedule_gloo_world2"}
            emit(out)
        return
    # per-step state in NB buffers: the discovery of step i writes coefs[i % NB] while older rollouts may
    # still read theirs (G|b and the gram workspace are only touched by the discovery stream, in order,
    # but are buffered alike to keep the plans independent).  Steps go in batches of K: one event per batch
    # each way (an event record costs ~20 us of dead queue time on ROCm 7.2, profiles/
    # r02/c2_pipeline_trace.txt); batches alternate between RS rollout streams and y buffers.
    K, RS = args.pipe_k, args.pipe_rs
    WAR_EVERY = 2 * K
    NB = 3 * K * RS                     # a multiple of K * RS: step k's y buffer (k // K) % RS is fixed per coef slot
    NBE = NB // K                       # event slots (batches in flight)
    # G|b of K consecutive steps in one flat bucket: at N > 1 the pipeline all-reduces a batch's K systems in
    # ONE collective (the ~1 KB all-reduce is latency-bound: once per batch, not once per step)
    buckets = [idist.MomentBucket(K, 2, F, dev) for _ in range(NB // K)]
    bufs = [buckets[j // K].bufs[j % K] for j in range(NB)]
    coefs = [torch.empty((2, F), dtype=torch.float64, device=dev) for _ in range(NB)]
    masks = [torch.empty((2, F), dtype=torch.int8, device=dev) for _ in range(NB)]
    iters = [torch.empty((2,), dtype=torch.int32, device=dev) for _ in range(NB)]
    mask = masks[0]
    wss = [ops.Workspace() for _ in range(NB)]
    mode = args.mode if (world == 1 or args.mode != "graph") else "seq"   # RCCL stays outside graphs
    if mode != "pipeline":
        RS = 1
    if mode != "pipeline":
        K = 1
    ys = [torch.empty((T, N) if args.layout == "time" else (N, T), dtype=torch.float64, device=dev)
          for _ in range(RS)]
    y = ys[0]
    s_g = torch.cuda.current_stream(dev)
    s_rs = [torch.cuda.Stream(dev) if mode == "pipeline" else s_g for _ in range(RS)]

    # one step = discovery (Gram -> [RCCL all-reduce when N > 1] -> STLSQ) then the rollout with that
    # step's coefficients.  Launches go through prepared plans (arguments validated and packed once).
    #   pipeline : discovery stream (gram with its in-launch reduction to G|b, [all-reduce,] STLSQ: no
    #              cross-stream hop inside it) | RS rollout streams taking alternate batches of K steps —
    #              NB-buffered coefficients; a batch's rollouts wait for one event after its last discovery,
    #              and the discovery stream waits, every WAR_EVERY steps, for the rollout batches whose
    #              buffers the next WAR_EVERY steps reuse.  Event records cost ~20 us of dead queue time
    #              each on ROCm 7.2 (profiles/r02/c2_pipeline_trace.txt), so there is one per batch per
    #              stream; every step still runs its own discovery and the rollout with its coefficients
    #   seq      : gram + in-launch reduction + STLSQ (N = 1) then the rollout, eagerly on one stream
    #   graph    : the seq step captured once in a HIP graph and replayed (N = 1)
    # The timed region holds no timing events: per-kernel durations come from the separate
    # roofline pass below (isolated launches) and rocprofv3.
    with torch.cuda.stream(s_g):
        fused = [ops.plan_sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, 100, True, 2,
                                    "smoothed4", wss[j], out=(coefs[j], masks[j], iters[j], bufs[j].G, bufs[j].b),
                                    layout=args.layout) for j in range(NB)]
        gram_plans = [ops.plan_gram(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 2, "smoothed4", wss[j],
                                    out=(bufs[j].G, bufs[j].b), layout=args.layout) for j in range(NB)]
        stlsq_plans = [ops.plan_stlsq(bufs[j].G, bufs[j].b, 0.1, 0.5, 100, True, out=(coefs[j], masks[j], iters[j]))
                       for j in range(NB)]
    roll_plans = [ops.plan_rollout(y0, coh.u, arm_cf, coefs[j], lib, coh.dt, method=args.method, T=T,
                                   out=ys[(j // K) % RS], layout="time_bits" if roll_layout == "tile_bits" else roll_layout)
                  for j in range(NB)]
    # cross-stream ordering through the HIP runtime directly (torch's Event wrappers cost ~3-5 us of host
    # time each; at N > 1 the host also issues the all-reduce, and must stay ahead of a ~70 us step)
    hip = HipEvents()
    ev = {k: hip.create() for k in [(n, j) for n in "gr" for j in range(NBE)]}
    hs_g = s_g.cuda_stream
    done_r = [None] * NBE                   # (batch, rollout-done event) per event slot
    pending = []                            # steps discovered, rollouts not yet issued
    f_fast = [p.bind(s_g) for p in fused]
    g_fast = [p.bind(s_g) for p in gram_plans]
    c_fast = [p.bind(s_g) for p in stlsq_plans]
    r_fast = [p.bind(s_rs[(j // K) % RS]) for j, p in enumerate(roll_plans)]
    stl_roll = not collective and mode == "pipeline" and args.stlsq_stream == "rollout"
    c_roll = [p.bind(s_rs[(j // K) % RS]) for j, p in enumerate(stlsq_plans)] if stl_roll else None

    def discover(i, st):
        """Discovery of step i on stream st (used by seq / graph and the roofline pass)."""
        j = i % NB
        if not collective:
            fused[j](st)
        else:
            gram_plans[j](st)
            with torch.cuda.stream(st):
                idist.reduce_moments(bufs[j])       # the only collective
            stlsq_plans[j](st)

    def step(i, tev=None):
        """One step; ``tev`` = (gram start, gram end, rollout start, rollout end) timing events recorded
        on the streams those kernels run on (the instrumented pass)."""
        j = i % NB
        if mode != "pipeline":                      # current stream: the capture stream under graph capture
            st = torch.cuda.current_stream(dev)
            if tev:
                hip.record(tev[0], st.cuda_stream)
            discover(i, st)
            if tev:
                hip.record(tev[1], st.cuda_stream)
                hip.record(tev[2], st.cuda_stream)
            roll_plans[j](st)
            if tev:
                hip.record(tev[3], st.cuda_stream)
            return
        if i % WAR_EVERY == 0:
            # steps i .. i+WAR_EVERY-1 reuse the buffers of steps i-NB .. bound: wait, on each rollout
            # stream, for its newest batch at or below bound's batch (a stream runs its batches in order;
            # NB >= WAR_EVERY + K, so that batch has been issued)
            bb = (i - NB + WAR_EVERY - 1) // K
            for r in range(RS):
                b = bb - ((bb - r) % RS)
                if b >= 0 and done_r[b % NBE] is not None and done_r[b % NBE][0] == b:
                    hip.wait(hs_g, done_r[b % NBE][1])
        if tev and i % K == 0:
            hip.record(tev[0], hs_g)
        if stl_roll:
            g_fast[j]()                             # gram + in-launch reduction (STLSQ: rollout stream)
        elif not collective:
            f_fast[j]()                             # gram + in-launch reduction, STLSQ
        else:
            g_fast[j]()                             # gram; the batch's all-reduce + STLSQs in flush()
        pending.append(i)
        if i % K == K - 1:
            flush(tev)

    def flush(tev=None):
        """Issue the rollouts of the pending batch behind one event on the discovery stream."""
        if not pending:
            return
        b = pending[0] // K
        if collective:                              # the batch's K systems: one collective, then K STLSQs
            with torch.cuda.stream(s_g):
                idist.reduce_bucket(buckets[(pending[0] % NB) // K], force=args.force_collective)  # the only collective
            for k in pending:
                c_fast[k % NB]()
        if tev:
            hip.record(tev[1], hs_g)
        hip.record(ev["g", b % NBE], hs_g)
        hs_r = s_rs[b % RS].cuda_stream
        hip.wait(hs_r, ev["g", b % NBE])
        if tev:
            hip.record(tev[2], hs_r)
        for k in pending:
            if stl_roll:
                c_roll[k % NB]()
            r_fast[k % NB]()
        if tev:
            hip.record(tev[3], hs_r)
        hip.record(ev["r", b % NBE], hs_r)
        done_r[b % NBE] = (b, ev["r", b % NBE])
        pending.clear()

    graph = None
    if mode == "graph":
        for i in range(2):                          # warm the plans outside capture
            step(i)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step(0)
        run = lambda i: graph.replay()  # noqa: E731
    else:
        run = step
    for i in range(args.warmup):
        run(i)
    if mode == "pipeline":
        flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        run(i)
    if mode == "pipeline":
        flush()                                     # a partial last batch
    host_ms = (time.perf_counter() - t0) / args.steps * 1e3   # submit time per step (no sync)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = idist.max_over_ranks(time.perf_counter() - t0, dev)
    ms_step = el / args.steps * 1e3
    coef = coefs[0] if mode == "graph" else coefs[(args.steps - 1) % NB]
    mask = masks[0] if mode == "graph" else masks[(args.steps - 1) % NB]

    # instrumented pass (after the timed region): the same schedule again — same streams, same overlap —
    # with HIP timing events around the gram and rollout launches on the streams they run on.  Per-launch
    # averages of the kernels exactly as they run in the step; a rocprofv3 --kernel-trace --stats run of
    # this bench (--no-north-star) averages the same pipelined launches (profiles/).
    n_inst = max(args.steps, 10) // K * K
    tevs = [tuple(hip.create(timing=True) for _ in range(4)) for _ in range(n_inst // K)]
    if mode == "graph":
        for i in range(n_inst):
            hip.record(tevs[i][0], torch.cuda.current_stream(dev).cuda_stream)
            graph.replay()
            hip.record(tevs[i][3], torch.cuda.current_stream(dev).cuda_stream)
    else:
        base = (args.steps + K - 1) // K * K       # start on a batch boundary (the timed run flushed its tail)
        for i in range(n_inst):
            step(base + i, tevs[i // K])
    torch.cuda.synchronize(dev)
    if mode == "graph":
        roll_ms = disc_ms = float(np.mean([hip.elapsed_ms(t[0], t[3]) for t in tevs]))
    else:                                           # per batch of K, divided by K
        disc_ms = float(np.mean([hip.elapsed_ms(t[0], t[1]) for t in tevs])) / K
        roll_ms = float(np.mean([hip.elapsed_ms(t[2], t[3]) for t in tevs])) / K

    # isolated launches (reported beside it, not as the roofline): each kernel back to back on one stream
    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st = torch.cuda.current_stream(dev)
        e0.record(st)
        for _ in range(n):
            fn(st)
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    iso = None
    if args.isolated:
        iso = {"rollout_avg_launch_ms": timed(roll_plans[0], n_inst),
               "gram_avg_launch_ms": timed(gram_plans[0], n_inst)}

    # sanity on the measured result: discovered support is the EQ_4_C one, no NaN
    sup = mask.cpu().numpy()
    ok = bool(torch.isfinite(y).all().item())

    out = None
    if rank == 0:
        arm_bits = 1 if roll_layout in ("time_bits", "tile_bits") else 8
        rb = rollout_bytes(N, T, arm_bits=arm_bits)
        achieved = rb / (roll_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                if tj.get("workload") == f"rollout_{args.method}_{N}x{T}":
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": METRIC,
            "value": N * world / (ms_step * 1e-3),
            "unit": "patient-trajectories/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: on-device EQ_4_C PK/PD cohort (reference distributions, Euler-5 truth + 0.01 noise)",
            "config": {
                "workload": f"C2: PK/PD {N // 1000}k patients/GPU x {T} steps fp64 - discovery (savgol+FD4+poly2 "
                            f"library+Gram, RCCL all-reduce when N>1, STLSQ) + {args.method.upper()} counterfactual rollout",
                "patients_per_gpu": N, "T": T, "rows_per_patient": T - 2, "library_terms": F,
                "parallelism": f"patient-shard x{world}" + (" (single-rank RCCL group: --force-collective)"
                                                             if args.force_collective and world == 1 else ""),
                "mode": mode, "stlsq_stream": "rollout" if stl_roll else "discovery",
                "discovered_support": sup.tolist(), "finite": ok,
            },
            "host_submit_ms_per_step": host_ms,
            "roofline": {
                "kernel": f"rollout_tm_kernel ({args.method})" if args.layout == "time" else f"rollout_kernel ({args.method})",
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": rb,
                "avg_launch_ms": roll_ms,
                "avg_ms_source": "instrumented pass: the timed schedule replayed with HIP timing events around "
                                 "each batch of rollout launches on its stream, divided by the batch size "
                                 "(concurrent with the next batch's discoveries)",
                "layout": {"time_bits": "time-major x[T,N], 1-bit arm mask [T,N/32], y[T,N]",
                           "tile_bits": "time-major x[T,N], 1-bit arm mask tile-major [N/64,T,2], y[T,N]",
                           "time": "time-major x[T,N], int8 arm[T,N], y[T,N]",
                           "patient": "patient-major x[N,T], int8 arm[N,T], y[N,T]"}[roll_layout],
            },
            "discovery": {
                "kernels": "gram_kernel (in-launch reduction to G|b, STLSQ in its last block)" if world == 1
                           else "gram_kernel (in-launch reduction) + RCCL all_reduce + stlsq_kernel",
                "timed_region": {"graph": "one step (gram+reduction, STLSQ, rollout) captured in a HIP graph, replayed",
                                 "seq": "eager launches, one stream, strictly sequential",
                                 "pipeline": f"discovery stream (gram+in-launch reduction [N>1: one all-reduce per "
                                             f"batch] +STLSQ) | {args.pipe_rs} rollout streams taking alternate "
                                             f"batches of {args.pipe_k} steps, one event per batch per stream, "
                                             f"{3 * args.pipe_k * args.pipe_rs} coefficient buffers"}[mode],
                "avg_ms_source": "instrumented pass: HIP timing events around each batch's discoveries (gram with its "
                                 "in-launch reduction, STLSQ) on their stream, divided by the batch size, "
                                 "concurrent with the previous batch's rollouts" if mode == "pipeline"
                                 else "instrumented pass: HIP timing events around discovery",
                "avg_ms": disc_ms,
                "algorithmic_bytes": gram_bytes(N, T),
                "achieved_GBps": gram_bytes(N, T) / (disc_ms * 1e-3) / 1e9,
                "frac": gram_bytes(N, T) / (disc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            },
            # both kernels share HBM inside a step: the step's whole algorithmic traffic over its time
            "step_aggregate": {"algorithmic_bytes": rb + gram_bytes(N, T),
                               "achieved_GBps": (rb + gram_bytes(N, T)) / (ms_step * 1e-3) / 1e9,
                               "frac": (rb + gram_bytes(N, T)) / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS},
        }
        if collective:
            # the bucketed all-reduce alone: back-to-back collectives on the discovery stream, HIP events around
            # the batch (per-collective device time incl. the process group's stream handshakes)
            fb = buckets[0].flat
            nc = 200
            with torch.cuda.stream(s_g):
                for _ in range(10):
                    idist.reduce_bucket(buckets[0], force=args.force_collective)
                torch.cuda.synchronize(dev)
                e0, e1 = hip.create(timing=True), hip.create(timing=True)
                t1 = time.perf_counter()
                hip.record(e0, hs_g)
                for _ in range(nc):
                    idist.reduce_bucket(buckets[0], force=args.force_collective)
                hip.record(e1, hs_g)
                torch.cuda.synchronize(dev)
                host_us = (time.perf_counter() - t1) / nc * 1e6
            out["collective"] = {"op": "all_reduce(SUM) of one batch bucket (RCCL)", "bytes": fb.numel() * 8,
                                 "systems_per_collective": K, "ranks": world,
                                 "avg_device_us": hip.elapsed_ms(e0, e1) / nc * 1e3, "avg_host_us": host_us,
                                 "per_step_us": hip.elapsed_ms(e0, e1) / nc * 1e3 / K}
        if iso is not None:
            out["isolated"] = dict(iso, rollout_frac=rb / (iso["rollout_avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                                   gram_frac=gram_bytes(N, T) / (iso["gram_avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS)
    # the same step as ONE fused launch (step_kernel, insite_fit_rollout_f64), measured beside the headline
    if rank == 0 and world == 1 and mode == "pipeline" and not args.no_fused:
        try:
            fr = fused_run(args, dev, coh, arm_cf)
        except Exception as exc:  # a secondary measurement never costs the headline line
            fr = None
            out["fused_step_kernel"] = {"error": f"{type(exc).__name__}: {exc}"}
    if rank == 0 and world == 1 and mode == "pipeline" and not args.no_fused and fr is not None:
        out["fused_step_kernel"] = {
            "kernel": "step_kernel (discovery of step i | rollout of step i-1, one launch per step)",
            "ms_per_step": fr["ms_step"], "avg_launch_ms": fr["step_ms"],
            "algorithmic_bytes_per_launch": fr["rb"] + fr["gb"],
            "achieved_GBps": (fr["rb"] + fr["gb"]) / (fr["step_ms"] * 1e-3) / 1e9, "frac": fr["frac"],
            "gram_blocks": args.gram_blocks or "default", "traffic": step_traffic(args),
            "avg_ms_source": f"HIP timing events around {fr['NBAT']} batches of {fr['KB']} back-to-back launches",
            "why_not_headline": "one launch holds both roles at the gram's 2 waves/SIMD register budget, the two-stream "
                                "pipeline keeps more rollout waves resident: the two measure within a few % of each "
                                "other, the pipeline ahead on most boxes (profiles/r02/fused_sweep/)",
        }
        del fr
    # the oracle parity of the benched cohort (every step of these modes discovers and rolls out the same cohort)
    if rank == 0 and world == 1 and not args.no_parity:
        out["parity"] = (c2_parity(dev, coh, arm_cf, coef, mask, y) if roll_layout in ("time_bits", "tile_bits") else
                         {"skipped": "the parity block reads the time-major bit-arm layout"})
    # north-star probe: 1M x 500 RK4 rollout alone (the >= 40 % roofline target), rank 0, N = 1
    if rank == 0 and world == 1 and not args.no_north_star:
        del y
        torch.cuda.empty_cache()
        out["north_star_rollout"] = north_star_rollout(args, dev, coef, lib)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        emit(out)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
