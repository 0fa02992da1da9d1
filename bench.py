#!/usr/bin/env python3
"""Benchmark: vectors quantized/sec of the 3-level RQ encode (512-d, [128,128,256]) on MI355X.

Workload (BASELINE.json configs[2], the largest single-GPU config): 10M x 512 fp32
synthetic song vectors per GPU (Gaussian mixture, generated on the device), PROD
codebooks (layer_clusters [128,1280,1280], need [128,128,256]: C1 128 x 512,
C2 16384 x 512, C3 2560 x 512 + a 16384 x 2560 match matrix with 256 allowed
columns per (l1,l2) group), training-consistent encode semantics (exact argmin,
normalised residuals).  A step = one full 3-level encode of the rank's batch,
inputs resident in HBM.  Multi-GPU: one process per GPU, rows sharded (weak
scaling: every rank encodes its own 10M rows), no data-path collective; the
timed region is bracketed by barrier + synchronize and the max over ranks is
taken.

Extra fields: ``roofline`` for the dominant kernel (per-launch time from HIP
events on the launch stream inside the timed region), ``kernels`` (per-level
breakdown), ``cpu_baseline`` (the oracle's CPU encode timed on this host on a
bounded sample, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from generative_ranking_recommender_amd import ops, synth  # noqa: E402
from generative_ranking_recommender_amd.distributed import Comm  # noqa: E402
from generative_ranking_recommender_amd.encode import HIERARCHICAL_TRAIN  # noqa: E402
from generative_ranking_recommender_amd.hierarchical_rq_kmeans import (  # noqa: E402
    HierarchicalRQKMeans, HierarchicalRQKMeansConfig)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA spec
D = 512
NEED = [128, 128, 256]
N_CAND = 2560


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preset", choices=("prod", "xl"), default="prod",
                    help="prod: need [128,128,256], 2560 last-level candidates (BASELINE configs[2]/[3], the "
                         "headline); xl: need [256,256,512], 5120 candidates (configs[4]: 50M rows over 8 GPUs = "
                         "6.25M rows per GPU by default)")
    ap.add_argument("--rows", type=int, default=0, help="rows per GPU (0: 10M for prod, 6.25M for xl)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="rows for the CPU baseline (0 = skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--codebooks", choices=("fitted", "sampled"), default=os.environ.get("BENCH_CODEBOOKS", "fitted"),
                    help="fitted: short K-Means fits on a sample (trained-model geometry); sampled: residual rows")
    ap.add_argument("--traffic-json", default=str(REPO / "bench_data" / "traffic.json"),
                    help="PMC HBM bytes per launch of this build (tools/pmc_traffic.sh; shipped to the GPU box, "
                         "unlike profiles/); missing file -> traffic null")
    ap.add_argument("--balanced-rows", type=int, default=1000000,
                    help="rows of the balanced (auction) training iterations in 'train_balanced' (0 = skip)")
    ap.add_argument("--train-iters", type=int, default=3,
                    help="Lloyd iterations timed for the 'train' field (0 = skip)")
    ap.add_argument("--side-budget", type=float, default=0.0,
                    help="seconds the side measurements after the timed region may take before the encode line is "
                         "printed without the rest and every rank exits (0: 600 at N=1, 300 at N>1)")
    ap.add_argument("--config0", type=int, default=1,
                    help="1: also run BASELINE configs[0] (100k, single level K=128, simplified path) on the GPU and "
                         "its CPU restatement on a bounded sample (field 'config0')")
    ap.add_argument("--parity-rows", type=int, default=2048,
                    help="rows of the timed output checked against the exact CPU oracle after the run (0 = skip)")
    a = ap.parse_args()
    global NEED, N_CAND, PRESET
    PRESET = a.preset
    if a.preset == "xl":
        NEED, N_CAND = [256, 256, 512], 5120
        if a.traffic_json == str(REPO / "bench_data" / "traffic.json"):
            a.traffic_json = str(REPO / "bench_data" / "traffic_xl.json")
    if a.rows <= 0:
        a.rows = 6_250_000 if a.preset == "xl" else 10_000_000
    return a


# kernels of each encode level's rqsid_assign call under the default dispatch (assign.hip rqsid_assign:
# screen + exact re-score), per preset
LEVEL_KERNELS = {
    "prod": {0: ("assign_screen_kernel<4, 2, 0, false, false, true, 1>", "assign_rescore_half_kernel<0, false>"),
             1: ("assign_screen_kernel<4, 2, 1, true, true, true, 1>", "assign_rescore_half_kernel<1, true>"),
             2: ("assign_pc_kernel<8, 2, true, false>", "assign_rescore_half_kernel<2, true>")},
    # [256,256,512]: 256-candidate level 0 (per-tile form); 256-candidate 3-term level 1 in one pass
    # (candidate-split screen, CW = 2); 512-candidate level 2 on the row-resident screen (assign_rows.hip)
    "xl": {0: ("assign_screen_kernel<8, 2, 0, false, false, true, 1>", "assign_rescore_half_kernel<0, false>"),
           1: ("assign_screen_kernel<4, 2, 1, true, true, true, 2>", "assign_rescore_half_kernel<1, true>"),
           2: ("assign_rows_kernel<4, 4, 3, 2, 2, true>", "assign_rescore_half_kernel<2, true>")}}
PRESET = "prod"


def level_traffic(path, lvl, rows):
    """HBM bytes (PMC FETCH_SIZE x2 + WRITE_SIZE) of one launch of level lvl's kernels, or None -- also
    when the counters were collected at another row count than this run's (they do not scale exactly)."""
    try:
        d = json.load(open(path))
        if int(d.get("rows") or -1) != int(rows):
            return None
        ks = d["kernels"]
        return sum(ks[k]["hbm_bytes"] for k in LEVEL_KERNELS[PRESET][lvl])
    except (OSError, KeyError, TypeError, ValueError):
        return None


class SideWatchdog:
    """The encode line is complete before the side measurements (train / balanced / parity / config0 /
    CPU baseline) run, and those run collectives at N > 1.  If they take longer than ``budget`` seconds,
    rank 0 prints the encode line as measured so far (marked ``side_measurements: stopped``) and every
    rank exits with status 3 -- a hang is a failure the driver sees, while the line it needs is printed.
    ``done(line)`` prints the full line instead (exactly one line either way)."""

    EXIT_CODE = 3

    def __init__(self, line: dict, budget: float, rank: int, exit_fn=os._exit):
        self.line, self.budget, self.rank, self.exit_fn = line, budget, rank, exit_fn
        self.printed, self.lock = threading.Event(), threading.Lock()
        self.thread = threading.Thread(target=self._run, daemon=True)

    def start(self):
        self.thread.start()
        return self

    def _run(self):
        if self.printed.wait(self.budget):
            return
        with self.lock:
            if self.printed.is_set():
                return
            self.printed.set()
            if self.rank == 0:
                try:
                    snap = dict(self.line)
                    snap["side_measurements"] = f"stopped after {self.budget:.0f} s (watchdog; exit status {self.EXIT_CODE})"
                    print(json.dumps(snap), flush=True)
                except Exception:
                    pass
            sys.stdout.flush()
            self.exit_fn(self.EXIT_CODE)

    def done(self) -> bool:
        """print the full line (rank 0); False when the watchdog already printed its snapshot"""
        with self.lock:
            if self.printed.is_set():
                return False
            if self.rank == 0:
                print(json.dumps(self.line), flush=True)
            self.printed.set()
            return True


class Timed:
    """HIP-event brackets recorded on torch's current stream (the stream every rqsid call uses)."""

    def __init__(self):
        self.pairs = {}

    def wrap(self, name, fn):
        def inner(*a, **k):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            out = fn(*a, **k)
            e.record()
            self.pairs.setdefault(name, []).append((s, e))
            return out
        return inner

    def mean_ms(self):
        return {k: float(np.mean([s.elapsed_time(e) for s, e in v])) for k, v in self.pairs.items()}


def make_rows(n, rank, device):
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    means = torch.from_numpy(synth.blob_means()).to(device)
    x = torch.empty((n, D), dtype=torch.float32, device=device)
    step = 1 << 20
    for i in range(0, n, step):
        m = min(step, n - i)
        lab = torch.randint(0, means.shape[0], (m,), device=device, generator=g)
        x[i:i + m] = means[lab] + 0.25 * torch.randn((m, D), device=device, generator=g)
    return x


def _lloyd(x, k, iters, gen):
    """Short unbalanced K-Means on the device (rqsid nearest + fp64 centroid sums); empty clusters
    keep their previous centre.  Initial centres: k distinct rows (with replacement when k > n)."""
    n = x.shape[0]
    if n >= k:
        init = torch.randperm(n, device=x.device, generator=gen)[:k]
    else:
        init = torch.randint(0, n, (k,), device=x.device, generator=gen)
    c = x[init].clone()
    for _ in range(iters):
        a = ops.nearest(x, ops.prepare_centers(c))
        c, _ = ops.centroid_update(x, a, k, c)
    return c


def fitted_codebooks(device, n_sample=1_000_000, seed=4321, iters=10):
    """PROD-shaped codebooks FITTED on a sample of the bench distribution (what a trained model's
    codebooks look like): C1 = K-Means(128) of the rows; C2 = per-parent K-Means(128) of the
    normalised level-1 residuals; C3 = K-Means(2560) of the normalised level-2 residuals; match row
    of an (l1,l2) group = the 256 candidates nearest the mean residual of the group's sample rows
    (random columns for groups with no sample rows).  Short Lloyd fits (``iters`` iterations,
    unbalanced): the geometry of trained centroids, not the reference's balanced training."""
    gen = torch.Generator(device=device).manual_seed(seed)
    x = make_rows(n_sample, 10_000 + seed, device)
    c0 = _lloyd(x, NEED[0], iters, gen)
    a0 = ops.nearest(x, ops.prepare_centers(c0))
    r1 = ops.residual(x, c0, a0, normalize=True)
    order = torch.argsort(a0, stable=True)
    cnt0 = torch.bincount(a0.long(), minlength=NEED[0]).cpu().tolist()
    c1 = torch.empty((NEED[0] * NEED[1], D), dtype=torch.float32, device=device)
    a1 = torch.empty(n_sample, dtype=torch.int32, device=device)
    start = 0
    for p in range(NEED[0]):
        rows = order[start:start + cnt0[p]]
        start += cnt0[p]
        sub = r1[rows] if len(rows) else r1[:1]
        cp = _lloyd(sub, NEED[1], iters, gen)
        c1[p * NEED[1]:(p + 1) * NEED[1]] = cp
        if len(rows):
            a1[rows] = ops.nearest(sub, ops.prepare_centers(cp)) + p * NEED[1]
    r2 = ops.residual(r1, c1, a1, normalize=True)
    c2 = _lloyd(r2, N_CAND, iters, gen)
    groups = NEED[0] * NEED[1]
    sums = torch.zeros((groups, D), dtype=torch.float32, device=device).index_add_(0, a1.long(), r2)
    cnt = torch.bincount(a1.long(), minlength=groups)
    means = sums / cnt.clamp(min=1).unsqueeze(1).float()
    near = torch.topk(ops.pairwise_distance(means.contiguous(), c2), NEED[2], dim=1, largest=False).indices
    rand = torch.argsort(torch.rand((groups, N_CAND), device=device, generator=gen), dim=1)[:, :NEED[2]]
    cols = torch.where((cnt > 0).unsqueeze(1), near, rand)
    match = torch.zeros((groups, N_CAND), dtype=torch.uint8, device=device).scatter_(1, cols, 1)
    return {"c0": c0.cpu().numpy(), "c1": c1.cpu().numpy(), "c2": c2.cpu().numpy(), "match": match.cpu().numpy()}


def codebooks(kind, device):
    if kind == "fitted":
        return fitted_codebooks(device)
    return synth.encode_codebooks(seed=99, need=tuple(NEED), n_cand=N_CAND)


def cpu_baseline(cb, rows):
    from threadpoolctl import threadpool_info
    from oracle import rq_oracle as O
    x = synth.mixture_rows(0, rows)
    t = time.perf_counter()
    O.encode(x, [cb["c0"], cb["c1"], cb["c2"]], NEED, cb["match"], residual_from_weighted=True)
    dt = time.perf_counter() - t
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    return {"value": rows / dt, "unit": "vectors/s", "cores": int(threads), "kind": "port",
            "sample": f"{rows} rows x 3 levels, oracle/rq_oracle.py encode (numpy fp32 BLAS, {threads} threads), "
                      f"{dt:.2f} s"}


def _gpu_seconds(fn, reps=3):
    """Mean wall seconds of fn() on the device (synchronised), after one warm-up call."""
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def cpu_baselines_8d(cb, dev):
    """SURVEY §8(d)'s CPU-baseline set beside the same unit on the GPU, on the same rows (rank 0, N=1):
    single-level assign (K=128) at 100k and 1M rows, one Lloyd iteration (assign + centroid update) at 1M rows,
    one balanced-auction round at 100,001 x 128 (N % K != 0, as a 1002-round level-0 fit runs).  CPU: the
    oracle's restatements of the reference (balancekmeans/__init__.py:489-534 predict, :315-324 update,
    :12-140 auction with torch CPU ops); GPU: the librqsid path each replaces.  Bounded: ~10 s of CPU work."""
    from threadpoolctl import threadpool_info
    from oracle import rq_oracle as O
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    c0 = cb["c0"]
    c0d = torch.from_numpy(c0).to(dev)
    pc0 = ops.prepare_centers(c0d)
    out = {"cores": int(threads), "torch_threads": int(torch.get_num_threads()), "kind": "port",
           "note": "cpu: oracle/rq_oracle.py (numpy fp32 BLAS / torch CPU ops); gpu: librqsid on the same rows"}
    x1m = synth.mixture_rows(0, 1_000_000)
    for rows in (100_000, 1_000_000):
        xs = x1m[:rows]
        t = time.perf_counter()
        O.nearest(xs, c0)
        cpu = time.perf_counter() - t
        xd = torch.from_numpy(xs).to(dev)
        gpu = _gpu_seconds(lambda: ops.nearest(xd, pc0))
        out[f"assign_k128_{rows // 1000}k"] = {
            "unit": "rows/s", "cpu": round(rows / cpu, 1), "gpu": round(rows / gpu, 1),
            "cpu_s": round(cpu, 3), "gpu_ms": round(gpu * 1e3, 3),
            "reference": "balancekmeans/__init__.py:489-534 (pairwise_distance_full + argmin)"}
    # one Lloyd iteration (unbalanced KMeans.fit step) at 1M rows
    t = time.perf_counter()
    a = O.nearest(x1m, c0)
    O.centroid_update(x1m, a, c0, lambda n: 0)
    cpu = time.perf_counter() - t
    xd = torch.from_numpy(x1m).to(dev)

    def lloyd():
        ids = ops.nearest(xd, ops.prepare_centers(c0d))
        ops.centroid_update(xd, ids, c0.shape[0], c0d.clone())
    gpu = _gpu_seconds(lloyd)
    out["lloyd_iteration_1m"] = {"unit": "rows/s", "cpu": round(1e6 / cpu, 1), "gpu": round(1e6 / gpu, 1),
                                 "cpu_s": round(cpu, 3), "gpu_ms": round(gpu * 1e3, 3),
                                 "reference": "balancekmeans/__init__.py:368-465 (one fit iteration: predict + :315-324)"}
    # one balanced-auction round at 100,001 jobs x 128 workers
    n_a = 100_001
    d = O.cdist_f32(x1m[:n_a], c0)
    rounds_cpu = 5
    cpu_round = O.auction_rounds_torch_cpu(-d, rounds_cpu)
    w = torch.from_numpy(np.ascontiguousarray((-d).T)).to(dev).half().contiguous()
    ops.auction(w)
    torch.cuda.synchronize()
    t = time.perf_counter()
    _, r = ops.auction(w)
    torch.cuda.synchronize()
    g = time.perf_counter() - t
    rounds = int(r) if not isinstance(r, torch.Tensor) else int(r.max().item())
    out["auction_round_100k"] = {"unit": "ms per round", "cpu": round(cpu_round * 1e3, 3),
                                 "gpu": round(g / max(rounds, 1) * 1e3, 4),
                                 "sample": f"{n_a} x 128 fp16 scores; cpu: {rounds_cpu} rounds of the reference's "
                                           f"torch CPU ops; gpu: the whole auction ({rounds} rounds) / rounds",
                                 "reference": "balancekmeans/__init__.py:12-140 (auction_lap_half)"}
    return out


def config0(dev, rows=100_000, cpu_rounds=40):
    """BASELINE configs[0]: 100k x 512, single level K=128, the simplified path (simplified_semantic_id_
    generator.py:176-245 with layer_clusters = need = [128]: one balanced fit_by_min_loss with target
    np.prod([]) = 1.0 (Appendix A item 9), then predict).  GPU: the whole SimplifiedHierarchicalRQ.train
    on the HIP path (train_rows: rows already loaded).  CPU: the oracle's restatement of one Lloyd
    iteration of that fit (fp32 cdist + auction_lap_half + update) timed on a bounded sample of
    ``cpu_rounds`` auction rounds and scaled to the iteration's rounds (1002 here: N % K != 0)."""
    from generative_ranking_recommender_amd.simplified_semantic_id_generator import SimplifiedHierarchicalRQ
    from oracle import rq_oracle as O
    xs = synth.mixture_rows(0, rows)
    cfg = HierarchicalRQKMeansConfig(layer_clusters=[128], need_clusters=[128], embedding_dim=D)
    m = SimplifiedHierarchicalRQ(cfg, device=dev)
    np.random.seed(42)
    torch.manual_seed(42)
    sids = [str(i) for i in range(rows)]
    torch.cuda.synchronize()
    t = time.perf_counter()
    m.train_rows(sids, torch.from_numpy(xs))
    torch.cuda.synchronize()
    gpu_s = time.perf_counter() - t
    km = m.trained_kmeans_models[0]
    iters = len(km.last_auction_rounds)
    ids = np.array([m.semantic_ids[s][0] for s in sids])
    # parity: every song's id is the exact nearest trained centre (the oracle on an evenly spaced sample)
    # and the fit's balance is the reference's (:197: target 1.0 -> every cluster over-full, the min-loss
    # choice falls on the latest iteration's centres)
    c = km.cluster_centers.detach().cpu().numpy()
    smp = np.linspace(0, rows - 1, 4096).astype(np.int64)
    want = O.nearest(xs[smp], c, exact=True)
    out = {"workload": f"SimplifiedHierarchicalRQ.train, {rows} x {D}, layer_clusters = need_clusters = [128], "
                       f"iter_limit {cfg.iter_limit} (BASELINE configs[0])",
           "gpu": {"seconds": round(gpu_s, 2), "iterations": iters,
                   "auction_rounds": int(np.sum(km.last_auction_rounds)),
                   "s_per_iteration": round(gpu_s / max(iters, 1), 4),
                   "ids_in_range": bool((ids >= 0).all() and (ids < 128).all())},
           "parity": {"rows_checked": int(len(smp)), "mismatches": int((ids[smp] != want).sum()),
                      "against": "oracle/rq_oracle.py nearest(exact=True) of the trained centres, evenly spaced rows",
                      "cluster_sizes_min_max": [int(np.bincount(ids, minlength=128).min()),
                                                int(np.bincount(ids, minlength=128).max())]}}
    if cpu_rounds <= 0:  # (tools/config0_time.py: the GPU fit alone)
        return out
    # the CPU restatement of one iteration (the reference's own arithmetic, numpy)
    rng = np.random.default_rng(0)
    c = xs[rng.choice(rows, 128, replace=False)]
    t = time.perf_counter()
    d = O.cdist_f32(xs, c)
    t_d = time.perf_counter() - t
    t_r = O.auction_rounds_torch_cpu(-d, cpu_rounds)
    a = d.argmin(1)
    t = time.perf_counter()
    O.centroid_update(xs, a, c, lambda n: 0)
    t_u = time.perf_counter() - t
    rounds = int(round(out["gpu"]["auction_rounds"] / max(iters, 1)))  # the GPU fit's own rounds per iteration
    cpu_iter = t_d + rounds * t_r + t_u
    from threadpoolctl import threadpool_info
    threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    out["cpu_baseline"] = {"value": round(cpu_iter, 2), "unit": "s per balanced Lloyd iteration", "cores": int(threads),
                           "kind": "port",
                           "sample": f"oracle/rq_oracle.py: cdist {t_d:.2f} s (numpy) + {cpu_rounds} auction rounds "
                                     f"at {t_r * 1e3:.1f} ms (torch CPU ops, scaled to the GPU fit's {rounds} rounds per "
                                     f"iteration) + update {t_u:.2f} s; "
                                     f"{threads} BLAS threads, torch {torch.get_num_threads()} threads"}
    out["gpu_vs_cpu_per_iteration"] = round(cpu_iter / max(out["gpu"]["s_per_iteration"], 1e-9), 1)
    return out


def train_iterations(x, c0, iters, world, n_global):
    """§8(d)'s training unit: rows x Lloyd iterations at level 0 (K = 128, unbalanced KMeans.fit step,
    balancekmeans/__init__.py:368-465): exact assign (rqsid_assign) + fp64 per-cluster sums and counts
    (rqsid_centroid_accumulate) + the mean update; with N > 1 the sums go through one RCCL all_reduce of
    the fused [K*D + K] fp64 buffer (distributed.ShardedLloyd).  Timed after the encode, outside its
    timed region; returns (ms per iteration (max over ranks), rows per second over all ranks)."""
    from generative_ranking_recommender_amd.distributed import ShardedLloyd
    k = c0.shape[0]
    if world > 1:
        import torch.distributed as tdist
        lloyd = ShardedLloyd(k, x, n_global)

        def step(c):
            return lloyd.step(c)[0]
    else:
        def step(c):
            a = ops.nearest(x, ops.prepare_centers(c))
            return ops.centroid_update(x, a, k, c.clone())[0]
    c = c0.clone()
    c = step(c)  # warm-up (workspaces, LDS attributes)
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    t = time.perf_counter()
    for _ in range(iters):
        c = step(c)
    torch.cuda.synchronize()
    if world > 1:
        tdist.barrier()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=x.device)
    if world > 1:
        Comm().all_reduce(el, op=tdist.ReduceOp.MAX)
    dt = float(el.item())
    return dt / iters * 1e3, n_global * iters / dt


def balanced_iterations(x, cb, rows, world=1):
    """The reference's actual training step is balanced: one iteration = fp16 scores
    -distance + auction_lap_half + centroid update.  Times, on the first ``rows`` rows of this rank, one
    level-0 iteration (K = 128, one auction) and one middle-layer iteration of all 128 parents in lockstep
    (segments = the rows' level-0 parents, K = 128 each: rqsid_seg_auction_scores + rqsid_seg_auction_lap_half
    + the update over 128 x 128 clusters), outside the encode's timed region."""
    xs = x[:rows].contiguous()
    c0 = torch.from_numpy(cb["c0"]).to(x.device).float()
    c1 = torch.from_numpy(cb["c1"]).to(x.device).float()
    k = c0.shape[0]

    if world > 1:
        # row-sharded balanced step: the ranks' rows form one auction (distributed.ShardedAuction: two
        # histogram all_reduces, one all_gather and one count all_reduce per round over RCCL) and the
        # centroid sums one all_reduce
        import torch.distributed as tdist
        from generative_ranking_recommender_amd.distributed import GpuAuctionPasses, ShardedAuction

        def level0():
            w = ops.auction_scores(xs, c0, half=False)
            a, r = ShardedAuction().run(GpuAuctionPasses(w, rows * world), rows * world, k)
            sums, counts = ops.centroid_sums(xs, a.long(), k)
            buf = torch.cat([sums.reshape(-1), counts.to(sums.dtype)])
            Comm().all_reduce(buf)
            return r
    else:
        def level0():
            w = ops.auction_scores(xs, c0, half=False)
            a, r = ops.auction(w)
            ops.centroid_update(xs, a, k, c0.clone())
            return r

    ids = ops.nearest(xs, ops.prepare_centers(c0))
    xr = ops.residual(xs, c0, ids, normalize=True)
    order = torch.sort(ids.long(), stable=True)[1]
    sizes = torch.bincount(ids.long(), minlength=k).cpu().numpy()
    xo = xr[order].contiguous()
    lay = ops.SegmentLayout(sizes, x.device)
    kk = c1.shape[0] // k

    def middle():
        w = ops.seg_auction_scores(xo, c1, kk, lay)
        a, r = ops.seg_auction(w, kk, lay)
        ops.centroid_update(xo, lay.seg_of_row * kk + a.long(), k * kk, c1.clone())
        return int(r.max().item())

    out = {}
    for name, fn in (("level0", level0), ("middle_lockstep", middle)):
        fn()  # warm-up
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        if world > 1:
            import torch.distributed as tdist
            el = torch.tensor([dt], dtype=torch.float64, device=x.device)
            Comm().all_reduce(el, op=tdist.ReduceOp.MAX)
            dt = float(el.item())
        tot = rows * (world if name == "level0" else 1)
        out[name] = {"ms_per_iteration": round(dt * 1e3, 2), "auction_rounds": int(r), "rows": tot,
                     "rows_per_s": round(tot / dt, 1)}
    out["middle_lockstep"]["segments"] = int((sizes > 0).sum())
    out["level0"]["sharding"] = f"rows sharded x{world}, RCCL exchange per auction round" if world > 1 else "one GPU"
    out["middle_lockstep"]["sharding"] = "per rank (rank 0's rows)"
    out["metric"] = "balanced Lloyd iteration (fp16 scores + auction_lap_half + centroid update)"
    return out


def check_sample(x, out, cb, rows):
    """The timed run's last output on an evenly spaced row sample vs the exact oracle (the checker only,
    after the timed region): the IDs must be identical."""
    from oracle import rq_oracle as O
    idx = torch.linspace(0, x.shape[0] - 1, rows, device=x.device).long()
    xs = x[idx].cpu().numpy()
    got = out[idx].cpu().numpy()
    ref = O.encode(xs, [cb["c0"], cb["c1"], cb["c2"]], NEED, cb["match"], residual_from_weighted=True, exact=True)
    bad = int((got != ref).any(1).sum())
    return {"rows_checked": rows, "mismatches": bad, "against": "oracle/rq_oracle.py encode(exact=True), evenly spaced rows"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    import torch.distributed as tdist
    # RQSID_BENCH_BACKEND=gloo: a rehearsal of the N-rank path on fewer GPUs (ranks share devices round-robin,
    # host-staged collectives); the driver's multi-GPU runs use RCCL, one rank per GPU
    backend = os.environ.get("RQSID_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    if dist:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        tdist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    cb = codebooks(args.codebooks, dev)
    # the library entry point: a trained HierarchicalRQKMeans (row-sharded over the process group when N > 1)
    # whose encode_shard is the hot path of predict (training-consistent semantics, IDs stay on the device)
    model = HierarchicalRQKMeans(HierarchicalRQKMeansConfig(layer_clusters=[NEED[0], N_CAND // 2, N_CAND // 2],
                                                            need_clusters=list(NEED), embedding_dim=D),
                                 device=dev, group=tdist.group.WORLD if dist else None)
    model.cluster_centers_list = [torch.from_numpy(cb[k]).to(dev) for k in ("c0", "c1", "c2")]
    model.match_matrices = [cb["match"]]
    model.is_trained = True
    enc = model._encoder(reference_quirks=False)
    assert enc.sem == HIERARCHICAL_TRAIN
    n = args.rows
    x = make_rows(n, rank, dev)
    torch.cuda.synchronize()

    # instrument the kernels (events only; no host sync inside the timed region)
    timer = Timed()
    orig_assign, orig_res, orig_bucket = ops.assign, ops.residual, ops.bucket
    level = {"i": 0}

    def assign_hook(*a, **k):
        name = f"assign_l{level['i']}"
        level["i"] += 1
        return timer.wrap(name, orig_assign)(*a, **k)

    import generative_ranking_recommender_amd.encode as encmod

    for _ in range(args.warmup):
        enc.encode(x)
    torch.cuda.synchronize()
    rescored = []
    enc.encode(x, count_rescored=True)
    rescored = list(enc.last_rescored)

    encmod.ops.assign = assign_hook
    encmod.ops.residual = timer.wrap("residual", orig_res)
    encmod.ops.bucket = timer.wrap("bucket", orig_bucket)

    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        level["i"] = 0
        out = model.encode_shard(x)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    encmod.ops.assign, encmod.ops.residual, encmod.ops.bucket = orig_assign, orig_res, orig_bucket
    gather_ms = None
    if dist:  # outside the timed region: the int32 IDs of every rank to every rank (the jsonl writer's input)
        try:
            t_g = time.perf_counter()
            ids_all = model.gather_ids(out)
            torch.cuda.synchronize()
            gather_ms = (time.perf_counter() - t_g) * 1e3
            assert ids_all.shape[0] == n * world
            del ids_all
        except Exception as exc:  # a side measurement must not cost the encode line
            gather_ms = repr(exc)[:300]

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist:
        Comm().all_reduce(el, op=tdist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms = timer.mean_ms()

    # roofline of the dominant kernel (algorithmic bytes / flops per launch)
    bytes_row = D * 4 + 4
    kern = {}
    for lvl, keff in ((0, NEED[0]), (1, NEED[1]), (2, NEED[2])):
        t = ms.get(f"assign_l{lvl}")
        if t is None:
            continue
        gbs = n * bytes_row / (t * 1e-3) / 1e9
        tfl = n * 2 * keff * D / (t * 1e-3) / 1e12
        kern[f"assign_l{lvl}"] = {"ms": round(t, 3), "GB/s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                                  "fp32_equiv_TFLOP/s": round(tfl, 1),
                                  "mfma_f16_frac": round(tfl / BF16_PEAK_TFLOPS, 4),
                                  "rescored_rows": rescored[lvl] if lvl < len(rescored) else None}
    if "residual" in ms:
        t = ms["residual"]
        gbs = n * (3 * D * 4) / (t * 1e-3) / 1e9
        kern["residual"] = {"ms": round(t, 3), "GB/s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
    if "bucket" in ms:
        kern["bucket"] = {"ms": round(ms["bucket"], 3)}
    dom = max((k for k in kern if k.startswith("assign")), key=lambda k: kern[k]["ms"])
    dk = kern[dom]
    traffic = level_traffic(args.traffic_json, int(dom[-1]), n) if os.environ.get("RQSID_SCREEN_VARIANT", "0") == "0" else None
    # Which roof applies: the level's algorithmic intensity (2 K_eff D flop per 2052 B: 64-128 flop/B) puts
    # its fp16 MFMA time at <= 6 % of its HBM time at the two peaks, so HBM is the roof; the PMC traffic
    # (when present) says whether the kernel moves more than its algorithmic bytes.
    keff = NEED[int(dom[-1])]
    t_hbm = n * bytes_row / (HBM_PEAK_GBS * 1e9)
    t_mfma = n * 2 * keff * D / (BF16_PEAK_TFLOPS * 1e12)
    roof = {"kernel": dom + " (rqsid_assign: fp16 MFMA screen kernel + exact re-score kernel)",
            "bound": "hbm" if t_hbm >= t_mfma else "mfma",
            "bound_basis": f"algorithmic: {t_hbm * 1e3:.2f} ms of HBM at peak vs {t_mfma * 1e3:.3f} ms of fp16 MFMA at "
                           f"peak per launch" + (f"; PMC traffic = {traffic / (n * bytes_row):.3f} x the algorithmic bytes"
                                                 if traffic else "; no PMC traffic for this build"),
            "achieved": dk["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": dk["hbm_frac"],
            "traffic": traffic, "traffic_unit": "bytes per launch",
            "traffic_source": (os.path.relpath(args.traffic_json, REPO) + " (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                               "separate passes, same build and workload)") if traffic else
                              "none: no PMC file for this build and row count",
            "algorithmic_bytes": n * bytes_row, "bytes_per_row": bytes_row}

    total_rows = n * world * args.steps
    value = total_rows / elapsed
    line = {
        "metric": "vectors quantized/sec (3-level RQ, 512-d)",
        "value": round(value, 1),
        "unit": "vectors/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic Gaussian mixture (4096 blobs, sigma 0.25) generated on device; " +
                (f"{'PROD' if NEED[0] == 128 else 'XL'}-shaped codebooks (need {NEED}) " +
                 ("fitted on a 1M-row sample (short Lloyd fits, random init)" if args.codebooks == "fitted"
                  else "sampled from residual rows")),
        "config": {"workload": f"3-level RQ encode, {n} x {D} fp32 rows per GPU, need {NEED}, layer_clusters "
                               f"[{NEED[0]},{N_CAND // 2},{N_CAND // 2}] (BASELINE "
                               + ("configs[2]/[3])" if NEED[0] == 128 else "configs[4] encode shapes)"),
                   "rows_per_gpu": n, "dim": D, "need_clusters": NEED, "candidates_last_level": N_CAND,
                   "parallelism": f"rows sharded x{world}, no collective in the step",
                   "entry_point": "HierarchicalRQKMeans.encode_shard (the per-rank hot path of predict)",
                   "method": "fp16 MFMA screen (LDS-DMA ring) + fp64 re-score (exact argmin)"},
        "roofline": roof,
        "kernels": kern,
    }
    if gather_ms is not None:
        line["gather_ids_ms"] = round(gather_ms, 3) if isinstance(gather_ms, float) else {"error": gather_ms}
    # The encode line is complete here.  The side measurements below run collectives at N > 1; a hang
    # there must not cost the line (SideWatchdog).
    dog = SideWatchdog(line, args.side_budget or (600.0 if world == 1 else 300.0), rank).start()
    if args.train_iters > 0:
        try:
            t_ms, rps = train_iterations(x, torch.from_numpy(cb["c0"]).to(dev).float(), args.train_iters, world,
                                         n * world)
            line["train"] = {"metric": "rows x Lloyd iterations/sec (level 0, K=128: assign + fp64 centroid update"
                                       + (", RCCL all_reduce of the [K*D+K] sums" if world > 1 else "") + ")",
                             "value": round(rps, 1), "unit": "rows/s", "ms_per_iteration": round(t_ms, 3),
                             "iterations": args.train_iters, "rows": n * world}
        except Exception as exc:  # a side measurement must not cost the encode line
            line["train"] = {"error": repr(exc)[:300]}
    if args.balanced_rows > 0:
        try:
            line["train_balanced"] = balanced_iterations(x, cb, min(args.balanced_rows, n), world)
        except Exception as exc:  # a side measurement must not cost the encode line
            line["train_balanced"] = {"error": repr(exc)[:300]}
    if args.parity_rows > 0:
        line["parity"] = check_sample(x, out, cb, args.parity_rows)
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        line["cpu_baseline"] = cpu_baseline(cb, args.cpu_sample)
        try:
            line["cpu_baselines_8d"] = cpu_baselines_8d(cb, dev)
        except Exception as exc:  # a side measurement must not cost the encode line
            line["cpu_baselines_8d"] = {"error": repr(exc)[:300]}
    if rank == 0 and world == 1 and args.config0:
        try:
            line["config0"] = config0(dev)
        except Exception as exc:  # a side measurement must not cost the encode line
            line["config0"] = {"error": repr(exc)[:300]}
    if not dog.done():
        return
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
