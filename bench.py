"""Benchmark: EM iterations/s of PoissonGPLVMJump1D.fit_em at BASELINE config C3
(N=512 neurons, T=1e5 time bins, L=512 latent bins; tuning_lengthscale=10 -> 79
basis columns; movement_variance=1, p_move_to_jump=p_jump_to_move=0.01; Adam lr 0.01,
maxiter 1000, tol 1e-6) on synthetic spikes drawn from the model itself.

One "step" = one full EM iteration on the device: sufficient statistics + Adam M-step
+ tuning + emission + forward filter + backward smoother (core.py:650-676).

N GPUs (one process per GPU, torchrun): every rank runs an independent EM restart
(model_selection_helper.py:53-59: restarts differ only in the posterior init) on the
same data -- no data-path collective, weak scaling; value = restarts x iterations / max
wall time over ranks.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (N, T, L)
    "c1": (30, 1000, 100),
    "c2": (128, 10000, 256),
    "c3": (512, 100000, 512),
    "c5": (256, 50000, 256),
    "c4": (1024, 1000000, 1024),
}
PEAK_HBM_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
PEAK_FP32_TFLOPS = 157.3         # dense FP32 matrix / packed vector (spec)
PEAK_BF16_MFMA_TFLOPS = 2500.0   # dense bf16 MFMA (spec, no sparsity)
PEAK_I8_MFMA_TOPS = 5000.0       # dense int8 MFMA (= fp8 rate, spec)


def synth(N, T, L, ls=10.0, seed=0, rank=0):
    """Synthetic workload (BASELINE.md section 2 seeds) with a vectorised sampler."""
    from poor_man_gplvm_amd.gp_kernel import generate_basis, create_transition_prob_1d
    B = generate_basis(ls, L)
    W = np.random.default_rng(seed).normal(size=(B.shape[1], N))
    F = B.astype(np.float64) @ W
    tun = np.logaddexp(F, 0.0)
    K, _, A, _ = create_transition_prob_1d(L, 1.0, 0.01, 0.01)
    rng = np.random.default_rng(seed + 1)
    lat = np.empty(T, np.int64)
    d, l = 0, L // 2
    cK = np.cumsum(K, axis=2)
    u = rng.random((T, 2))
    for t in range(T):
        d = 1 if u[t, 0] < A[d, 1] else 0
        l = int(min(np.searchsorted(cK[d, l], u[t, 1] * cK[d, l, -1], side="right"), L - 1))
        lat[t] = l
    y = np.random.default_rng(seed + 2).poisson(tun[lat]).astype(np.float32)
    uu = np.random.default_rng(seed + 3 + rank).random((T, L)) * 0.1
    p = uu / uu.sum(1, keepdims=True)
    lp0 = np.log(p).astype(np.float32)
    W0 = np.random.default_rng(123).normal(size=W.shape).astype(np.float32)
    return y, B, W0, lp0


class LazyRows:
    """(T, K) array whose row blocks are generated on demand: rows [a, b) of block
    size `block` come from fn(block_index) -> (rows, K), seeded per block, so every
    rank of a time-sharded run materialises only its own (extended) slice."""

    def __init__(self, T, K, fn, block=10000):
        self.shape = (T, K)
        self.fn, self.block = fn, block

    def __getitem__(self, sl):
        a, b, _ = sl.indices(self.shape[0])
        parts = []
        for k in range(a // self.block, (b - 1) // self.block + 1):
            blk = self.fn(k)
            lo, hi = max(a, k * self.block) - k * self.block, min(b, (k + 1) * self.block) - k * self.block
            parts.append(blk[lo:hi])
        return np.concatenate(parts, 0)


def synth_long(N, T, L, ls=10.0, seed=0, block=10000):
    """synth() for long recordings (C4): the latent path is sampled whole (cheap), the
    spikes and the posterior init per 10k-step block with per-block seeds."""
    from poor_man_gplvm_amd.gp_kernel import generate_basis, create_transition_prob_1d
    B = generate_basis(ls, L)
    W = np.random.default_rng(seed).normal(size=(B.shape[1], N))
    tun = np.logaddexp(B.astype(np.float64) @ W, 0.0)
    K, _, A, _ = create_transition_prob_1d(L, 1.0, 0.01, 0.01)
    rng = np.random.default_rng(seed + 1)
    cK = np.cumsum(K, axis=2)
    u = rng.random((T, 2))
    lat = np.empty(T, np.int64)
    d, l = 0, L // 2
    for t in range(T):
        d = 1 if u[t, 0] < A[d, 1] else 0
        l = int(min(np.searchsorted(cK[d, l], u[t, 1] * cK[d, l, -1], side="right"), L - 1))
        lat[t] = l

    def spikes(k):
        sl = lat[k * block:(k + 1) * block]
        return np.random.default_rng([seed + 2, k]).poisson(tun[sl]).astype(np.float32)

    def post0(k):
        n = min(block, T - k * block)
        uu = np.random.default_rng([seed + 3, k]).random((n, L)) * 0.1
        return np.log(uu / uu.sum(1, keepdims=True)).astype(np.float32)

    W0 = np.random.default_rng(123).normal(size=W.shape).astype(np.float32)
    return LazyRows(T, N, spikes, block), B, W0, LazyRows(T, L, post0, block)


def cpu_threads():
    """Host threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS, 16 on the
    GPU box), else every core this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def cpu_baseline(N, T, L, adam_iters, t_sample=1024, adam_sample=20):
    """The reference's EM iteration in float32 on all host cores (torch-CPU restatement,
    oracle/cpu_reference_fp32.py: dense log-domain filter and smoother with the per-step
    joint accumulation of decoder.py:221, T*L*N emission, suff-stats, Adam bodies) timed
    on a bounded sample of the same workload and scaled to one full EM iteration."""
    import torch
    from oracle import cpu_reference_fp32 as R
    threads = cpu_threads()
    torch.set_num_threads(threads)
    y, B, W0, _ = synth(N, t_sample, L)
    yt = torch.as_tensor(y)
    Bt = torch.as_tensor(B.astype(np.float32))
    Wt = torch.as_tensor(W0)
    tun = torch.nn.functional.softplus(Bt @ Wt)
    logK, logA = R.transition_logs(L)
    R.em_iteration_sample(yt[:8], tun, Bt, Wt, logK, logA, 1)          # first-touch warm-up
    t0 = time.perf_counter()
    R.em_iteration_sample(yt, tun, Bt, Wt, logK, logA, 0)
    t_step = (time.perf_counter() - t0) / t_sample                       # s per time step
    yw, tw = torch.rand(L, N) * (T / L), torch.full((L,), T / L)
    t0 = time.perf_counter()
    R.adam_steps(Wt, Bt, yw, tw, adam_sample)
    t_body = (time.perf_counter() - t0) / adam_sample                    # s per Adam body
    total = T * t_step + adam_iters * t_body
    return {"value": 1.0 / total, "unit": "EM iters/s", "cores": threads, "kind": "port",
            "sample": (f"float32 torch-CPU restatement of the reference EM iteration (oracle/cpu_reference_fp32.py; "
                       f"dense log-domain filter + smoother with per-step joint accumulation, emission, "
                       f"suff-stats, Adam) on {threads} threads: {t_sample} time steps x (N={N}, L={L}) and "
                       f"{adam_sample} Adam bodies timed ({1e3 * t_step:.2f} ms/step, {1e3 * t_body:.2f} ms/body), "
                       f"scaled to T={T} and {adam_iters:.0f} Adam bodies (the GPU run's mean): "
                       f"{total:.0f} s per EM iteration")}


def load_pmc(config):
    """Per-kernel HBM bytes from this round's PMC summary (tools/gpu_pmc.sh), if any."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{config}.json")
        if os.path.exists(path):
            with open(path) as fh:
                return json.load(fh).get("kernels", {}), os.path.relpath(path, ROOT)
    return {}, None


def fwdbwd_roofline(summ, T, L, pmc):
    """The metric's roofline: the forward-backward pair (main passes + verify/relaxation)
    against HBM, algorithmic bytes B_fb = 28*T*L per E-step: read the
    emission once, write and read back the filtered (T,2,L) state, write the posterior."""
    keys = ("forward_filter", "forward_repair", "backward_smoother", "backward_repair")
    t_ms = sum(summ[k][1] for k in keys if k in summ)
    B_fb = 28.0 * T * L
    achieved = B_fb / 1e9 / (t_ms / 1e3)
    traffic = None
    names = ("k_forward", "k_backward", "k_verify", "k_forward_relax", "k_backward_relax")
    if pmc and all(pmc.get(k, {}).get("hbm_bytes_per_launch") is not None for k in names[:2]):
        traffic = float(sum(pmc.get(k, {}).get("hbm_bytes_per_launch") or 0.0 for k in names))
    return {"kernel": "k_forward + k_backward (+ k_verify, k_forward_relax, k_backward_relax)",
            "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "ms_per_estep": round(t_ms, 4),
            "algorithmic_bytes_per_estep": B_fb}


def compute_rooflines(summ, T, L, N, NB, adam_iters, pmc):
    """Per-kernel rooflines (SURVEY.md 8(d) algorithmic units per launch) from the
    KernelTimer summary (HIP events on the launch stream).  T = time steps one launch
    processes.  The Adam loop is latency-bound by contract (a sequential stop rule over
    ~10 us f64-VALU bodies): it is reported per body, not against a throughput peak."""
    nblk = (L + 31) // 32
    units = {
        # section: (kernel, bound, algorithmic units per launch, unit scale, peak, unit)
        "forward_filter": ("k_forward", "hbm", 12.0 * T * L + 4.0 * T * nblk + 16.0 * T, 1e9, PEAK_HBM_GBS, "GB/s"),
        "backward_smoother": ("k_backward", "hbm", 16.0 * T * L + 4.0 * T * nblk, 1e9, PEAK_HBM_GBS, "GB/s"),
        "suffstats": ("k_ptb3", "mfma", 2.0 * T * L * N, 1e12, PEAK_BF16_MFMA_TFLOPS, "TFLOP/s"),
        "emission": ("k_emission_yreg" if N <= 512 else "k_emission_pipe", "mfma", 2.0 * T * L * N, 1e12,
                     PEAK_I8_MFMA_TOPS, "TOP/s"),
    }
    rooflines = {}
    for sec, (kname, bound, units_per_launch, scale, peak, unit) in units.items():
        if sec not in summ:
            continue
        t_ms = summ[sec][1]
        achieved = units_per_launch / scale / (t_ms / 1e3)
        tr = pmc.get(kname, {}).get("hbm_bytes_per_launch")
        rooflines[sec] = {"kernel": kname, "bound": bound, "achieved": achieved, "peak": peak, "unit": unit,
                          "frac": achieved / peak, "traffic": tr, "ms": round(t_ms, 4),
                          "algorithmic_per_launch": units_per_launch}
    if "mstep_adam" in summ:
        t_ms = summ["mstep_adam"][1]
        rooflines["mstep_adam"] = {"kernel": "k_adam", "bound": "latency (f64 VALU, sequential stop rule)",
                                   "ms": round(t_ms, 4), "bodies": adam_iters,
                                   "us_per_body": 1e3 * t_ms / max(adam_iters, 1.0)}
    return rooflines


def bench_timeshard(args):
    """One EM iteration of ONE recording time-sharded over the ranks (timeshard.py):
    value = EM iterations/s of the whole job (total T fixed: strong scaling)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    # RCCL whenever torchrun launched us (also at one rank: the DistComm / RCCL path of
    # the time shards then runs its collectives on device buffers), else virtual shards
    rccl = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if rccl:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()       # n_gpus = the world RCCL sees
    from poor_man_gplvm_amd.engine import AdamConfig, ScanConfig, KernelTimer
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    from poor_man_gplvm_amd.timeshard import DistComm, LocalComm, TimeShardedEM, shard_layout

    N, T, L = CONFIGS[args.config]
    t_syn = time.perf_counter()
    y, B, W0, lp0 = synth_long(N, T, L) if T > 200000 else synth(N, T, L)
    t_syn = time.perf_counter() - t_syn
    comm = DistComm() if rccl else LocalComm(args.virtual)
    scan = ScanConfig(chunk=args.chunk or None, warmup=args.warm_steps)
    lays = shard_layout(T, comm.world, chunk=args.chunk or None, halo=args.halo, scan=scan)
    eng = TimeShardedEM(y, B, banded_transition(L, 1.0, 0.01, 0.01), comm, lays, scan,
                        neuron_sharded=not args.replicated_adam)
    for s in eng.shards:
        s.set_log_posterior(np.asarray(lp0[s.lay.ext_start:s.lay.ext_stop]))
        if args.warm_fb:
            s.warm = [int(v) for v in args.warm_fb.split(",")]
    dev = eng.dev
    adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6, prior_std=1.0)
    n = len(eng.shards)
    Ws = [torch.as_tensor(W0.astype(np.float64), device=dev).contiguous() for _ in range(n)]
    mus = [torch.zeros_like(Ws[0]) for _ in range(n)]
    nus = [torch.zeros_like(Ws[0]) for _ in range(n)]
    cnts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(n)]
    n_all = args.warmup + args.steps
    n_inst = min(args.steps, 5)      # instrumented iterations after the timed window
    stats = torch.zeros((n_all + n_inst, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_all + n_inst, adam.maxiter), dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    logz = torch.zeros(n_all + n_inst, dtype=torch.float64, device=dev)
    rounds = []

    def em_iter(i):
        eng.m_step(Ws, mus, nus, cnts, adam, stats[i], lh[i], eh[i])
        eng.e_step(1.0, logz[i:i + 1])
        rounds.append(tuple(eng.carry_rounds))

    warm_s, it0 = [], None
    for i in range(args.warmup):
        t0 = time.perf_counter()
        if i == 0:
            t_first = KernelTimer()
            eng.set_timer(t_first)
        em_iter(i)
        torch.cuda.synchronize()
        warm_s.append(time.perf_counter() - t0)
        if i == 0:
            eng.set_timer(None)
            s0 = t_first.summary()
            it0 = {"wall_s": round(warm_s[0], 4),
                   "scans_ms": round(sum(s0[k][1] * s0[k][0] for k in ("forward_filter", "forward_repair",
                                                                        "backward_smoother", "backward_repair")
                                         if k in s0), 2),
                   "kernels_ms_total": {k: round(v[1] * v[0], 3) for k, v in s0.items()},
                   "repairs": [list(s.repairs()) for s in eng.shards]}
    torch.cuda.synchronize()
    eng.set_timer(None)          # the timed window runs uninstrumented (as the default engine's)
    if rccl:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, n_all):
        em_iter(i)
    torch.cuda.synchronize()
    if rccl:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if rccl:
        te = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = float(te.item())
    # per-section HIP events over a few more iterations of the same fit
    timer = KernelTimer()
    eng.set_timer(timer)
    for i in range(n_all, n_all + n_inst):
        em_iter(i)
    torch.cuda.synchronize()
    eng.set_timer(None)
    summ = timer.summary()      # mean per call; every local shard makes its own calls
    st = stats.cpu().numpy()
    adam_iters = float(np.mean(st[args.warmup:n_all, 0])) if args.steps else 0.0
    T_ext = max(s.T for s in eng.shards)
    pmc, pmc_src = load_pmc(args.config)
    rooflines = compute_rooflines(summ, T_ext, L, N, B.shape[1], adam_iters, pmc)
    roof_dom = fwdbwd_roofline(summ, T_ext, L, pmc)
    t_fb = summ["forward_filter"][1] + summ["backward_smoother"][1]
    out = {
        "metric": (f"EM iters/sec at {args.config.upper()} (N={N}, T={T}, L={L}), one recording time-sharded"
                   if args.config != "c3" else "EM iters/sec at N=512, T=1e5, B=512; fwd-bwd achieved HBM GB/s"),
        "value": args.steps / elapsed,
        "unit": "EM iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 state / int8-exact emission / f64 stats",
        "data": "synthetic (spikes sampled from the model; per-10k-block seeds for long recordings)",
        "config": {"workload": f"{args.config}: ONE PoissonGPLVMJump1D.fit_em N={N} T={T} L={L} nb={B.shape[1]}, "
                               f"time-sharded over {comm.world} shard(s) ({n} per process), halo {args.halo}; "
                               f"one EM iteration per step",
                   "n_neuron": N, "n_time": T, "n_latent_bin": L,
                   "parallelism": f"time shards x{comm.world} (RCCL all-reduce of y_w/t_w + carry send/recv"
                                  + (", neuron-sharded Adam)" if eng.neuron_sharded else ")")},
        "roofline": roof_dom,
        "rooflines": rooflines,
        "kernels_ms": {k: round(v[1], 4) for k, v in summ.items()},
        "kernels_ms_note": (f"per-section HIP events of {n_inst} more iterations of the same fit right after "
                            "the timed window (the timed iterations run without them)"),
        "fwd_bwd_GBps_per_shard": 28.0 * T_ext * L / 1e9 / (t_fb / 1e3),
        "adam_iters_mean": adam_iters,
        "chunk": lays[0].chunk,
        "carry_rounds_timed": rounds[args.warmup:n_all],
        "repairs_last": [list(s.repairs()) for s in eng.shards],
        "first_iteration": it0,
        "warmup_iteration_s": [round(v, 4) for v in warm_s],
        "synth_s": round(t_syn, 1),
    }
    out["comm"] = "rccl" if rccl else f"local x{args.virtual}"
    if rank == 0:
        print(json.dumps(out), flush=True)
    if rccl:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=19, help="timed EM iterations")
    ap.add_argument("--warmup", type=int, default=1, help="untimed leading EM iterations of the same fresh fit")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-api-fit", action="store_true", help="skip the public-API fit_em(n_iter=20) timing")
    ap.add_argument("--decode", action="store_true",
                    help="also time decode_latent at this config (exact dense and banded paths)")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--chunk-bwd", type=int, default=0, help="backward chunk (0: ScanConfig default, 2x forward)")
    ap.add_argument("--warm-steps", type=int, default=48)
    ap.add_argument("--two-waves", action="store_true", help="main-pass chains on two waves (PMG_PHASE_TWO_WAVES)")
    ap.add_argument("--scan-tol", type=float, default=0.0, help="boundary tolerance (0: ScanConfig default)")
    ap.add_argument("--warm-fb", type=str, default="", help="fixed forward,backward warm-up (no adaptation)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--shard", default="restarts", choices=["restarts", "time"],
                    help="multi-GPU axis: independent restarts (weak scaling) or time shards of one "
                         "recording (strong scaling, RCCL suff-stat all-reduce + carry hand-off)")
    ap.add_argument("--virtual", type=int, default=1, help="time shards per process (single-GPU rehearsal)")
    ap.add_argument("--halo", type=int, default=512, help="time-shard halo (steps)")
    ap.add_argument("--replicated-adam", action="store_true",
                    help="time shards: run the whole Adam loop on every rank instead of one neuron block each")
    ap.add_argument("--restarts", type=int, default=0,
                    help="R > 1: R restarts per GPU as one batched fit (engine.RestartBatchEM; SURVEY 8(e), "
                         "C5 runs 8 per GPU); reports restart-iterations/s beside the one-restart engine")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU-only check of the N-rank launcher: gloo ranks, barrier + max-over-ranks timing of "
                         "a host loop, one JSON line (no GPU is touched)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # N ranks requested without a launcher: start them as children (this process
        # never touches the GPU) and exit with their status
        return launch_ranks(args.gpus)
    if args.launcher_selftest:
        return launcher_selftest(args)
    if args.shard == "time":
        return bench_timeshard(args)
    if args.restarts > 1:
        return bench_restarts(args)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()       # n_gpus = the world RCCL sees

    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig, KernelTimer
    from poor_man_gplvm_amd.gp_kernel import banded_transition

    N, T, L = CONFIGS[args.config]
    y, B, W0, lp0 = synth(N, T, L, rank=rank)
    dev = torch.device("cuda", local)
    scan = ScanConfig(chunk=args.chunk or None, warmup=args.warm_steps, chunk_bwd=args.chunk_bwd or None,
                      two_waves=args.two_waves)
    if args.scan_tol > 0:
        scan.tol = args.scan_tol
    sp = SpikeData(y)
    eng = DeviceEM(sp, L, basis=B, scan=scan)
    eng.adaptive = True          # as run_em: adaptive warm-up across the fit's E-steps
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6, prior_std=1.0)
    W = torch.empty((B.shape[1], N), dtype=torch.float64, device=dev)
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    n_all = args.warmup + args.steps
    stats = torch.zeros((n_all, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_all, adam.maxiter), dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    logz = torch.zeros(n_all, dtype=torch.float64, device=dev)

    def fresh_fit():
        """Reset to the start of a fit: the initial posterior, W init, Adam state 0."""
        eng.set_log_posterior(lp0)
        eng.reset_adaptive()
        W.copy_(torch.as_tensor(W0.astype(np.float64), device=dev))
        mu.zero_()
        nu.zero_()
        cnt.zero_()
        eng.warm = [int(args.warm_steps), int(args.warm_steps)]
        if args.warm_fb:
            eng.warm = [int(v) for v in args.warm_fb.split(",")]

    def em_iter(i):
        eng.m_step(W, mu, nu, cnt, adam, stats[i], lh[i], eh[i])
        eng.compute_tuning(W)
        eng.e_step(1.0, logz[i:i + 1])

    # pre-warm: one iteration of a throwaway fit loads every kernel's code object
    fresh_fit()
    em_iter(0)
    torch.cuda.synchronize()
    def timed_fit(timer):
        """One fresh fit: iterations 0 .. W-1 untimed (each timed on its own for the report),
        then K timed iterations bracketed by barrier + synchronize; timer: per-section HIP
        event pairs (KernelTimer) or None."""
        fresh_fit()
        warm_s = []
        for i in range(args.warmup):
            t0 = time.perf_counter()
            em_iter(i)
            torch.cuda.synchronize()
            warm_s.append(time.perf_counter() - t0)
        eng.timer = timer
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.warmup, n_all):
            em_iter(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            te = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
            elapsed = float(te.item())
        eng.timer = None
        return elapsed, warm_s

    # the measured fit runs uninstrumented; an identical second fresh fit records the
    # per-section HIP events (kernels_ms, rooflines) -- 18 event records per iteration
    # are instrumentation, not workload
    elapsed, warm_s = timed_fit(None)
    timer = KernelTimer()
    elapsed_instrumented, _ = timed_fit(timer)
    eng.timer = None
    summ = timer.summary()
    s = stats.cpu().numpy()
    adam_iters = float(np.mean(s[args.warmup:, 0])) if args.steps else 0.0
    repairs = eng.repairs()
    relax_rounds = eng.relax_rounds()
    lz_host = logz.cpu().numpy()

    pmc, pmc_src = load_pmc(args.config)
    rooflines = compute_rooflines(summ, T, L, N, B.shape[1], adam_iters, pmc)
    roof = fwdbwd_roofline(summ, T, L, pmc)
    value = world * args.steps / elapsed
    fresh_s = sum(warm_s) + elapsed
    out = {
        "metric": "EM iters/sec at N=512, T=1e5, B=512; fwd-bwd achieved HBM GB/s",
        "value": value,
        "unit": "EM iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 state / int8-exact emission / f64 stats",
        "data": "synthetic (spikes sampled from the model; seeds of BASELINE.md section 2)",
        "config": {"workload": f"{args.config}: PoissonGPLVMJump1D.fit_em N={N} T={T} L={L} nb={B.shape[1]}; "
                               f"one step = one EM iteration of a fresh fit (timed: iterations "
                               f"{args.warmup + 1}..{n_all}, 1-based); ranks = independent restarts",
                   "n_neuron": N, "n_time": T, "n_latent_bin": L, "parallelism": f"restarts x{world}"},
        "roofline": roof,
        "rooflines": rooflines,
        "fresh_fit": {"iterations": n_all, "device_s": fresh_s, "em_iters_per_s": n_all / fresh_s,
                      "warmup_iteration_s": [round(v, 5) for v in warm_s],
                      "note": "device-resident EM iterations 1..W+K of one fresh fit (after a one-iteration "
                              "code-object pre-warm), W untimed ones synchronised one by one"},
        "kernels_ms": {k: round(v[1], 4) for k, v in summ.items()},
        "kernels_ms_note": "from a second, identical fresh fit with per-section HIP events (the measured fit "
                           "runs without them)",
        "ms_per_step_instrumented": 1e3 * elapsed_instrumented / args.steps,
        "kernel_calls": {k: v[0] for k, v in summ.items()},
        "adam_iters_mean": adam_iters,
        "chunk": eng.C,
        "chunk_bwd": eng.Cb,
        "scan_tol": eng.scan.tol,
        "repairs_last": repairs,
        "relax_rounds_last": relax_rounds,
        "scan_warmup_fwd_bwd": list(eng.warm),
        "log_marginal_last": float(lz_host[n_all - 1]),
        "pmc_source": pmc_src,
    }
    if rank == 0 and world == 1 and not args.no_api_fit:
        out["fit_em_api"] = api_fit_wall(y, B, W0, lp0, L)
    if rank == 0 and world == 1 and args.decode:
        out["decode_latent"] = decode_leg(y, eng.tuning64.cpu().numpy(), L)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(N, T, L, adam_iters)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_restarts(args):
    """R restarts of one recording per GPU (model_selection_helper.py:53-59; C5 = 64
    restarts over 8 GPUs = 8 per GPU): one step = one EM iteration of all R restarts as
    ONE batched fit (stacked-latent emission and suff-stats GEMMs, one scan launch per
    pass, R Adam loops).  value = R x steps / time (restart-iterations/s, summed over
    ranks).  The same R restarts run one after another on the single-restart engine
    are timed beside it (sequential_restart_iters_per_s)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()       # n_gpus = the world RCCL sees
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, RestartBatchEM, AdamConfig, ScanConfig, KernelTimer
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    cfg = args.config if args.config != "c3" else "c5"
    N, T, L = CONFIGS[cfg]
    R = args.restarts
    y, B, W0, _ = synth(N, T, L, rank=rank)
    lps = []
    for r in range(R):                      # restart r of rank k: posterior-init seed 3 + k R + r
        uu = np.random.default_rng(3 + rank * R + r).random((T, L)) * 0.1
        lps.append(np.log(uu / uu.sum(1, keepdims=True)).astype(np.float32))
    lps = np.stack(lps)
    dev = torch.device("cuda", local)
    adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6, prior_std=1.0)
    tr = banded_transition(L, 1.0, 0.01, 0.01)
    sp = SpikeData(y)
    n_all = args.warmup + args.steps
    eng = RestartBatchEM(sp, L, B, R, scan=ScanConfig(chunk=args.chunk or None, warmup=args.warm_steps))
    eng.set_transition(tr)
    NB = B.shape[1]
    W = torch.empty((R, NB, N), dtype=torch.float64, device=dev)
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(R, dtype=torch.int64, device=dev)
    stats = torch.zeros((n_all, R, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_all, R, adam.maxiter), dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    logz = torch.zeros((n_all, R), dtype=torch.float64, device=dev)

    def fresh():
        eng.set_log_posterior(lps)
        eng.reset_adaptive()
        W.copy_(torch.as_tensor(np.broadcast_to(W0.astype(np.float64), (R, NB, N)).copy(), device=dev))
        mu.zero_(); nu.zero_(); cnt.zero_()

    def it(i):
        eng.m_step(W, mu, nu, cnt, adam, stats[i], lh[i], eh[i])
        eng.compute_tuning(W)
        eng.e_step(1.0, logz[i])

    def run(fresh_fn, step_fn, timed_engine=None, timer=None):
        fresh_fn(); step_fn(0); torch.cuda.synchronize()     # code-object pre-warm
        fresh_fn()
        for i in range(args.warmup):
            step_fn(i)
        torch.cuda.synchronize()
        if timed_engine is not None:
            timed_engine.timer = timer
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.warmup, n_all):
            step_fn(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if timed_engine is not None:
            timed_engine.timer = None
        if world > 1:
            te = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
            el = float(te.item())
        return el
    timer = KernelTimer()
    elapsed = run(fresh, lambda i: it(i), eng, timer)      # per-kernel HIP events over the timed window
    summ = timer.summary()
    s = stats.cpu().numpy()
    adam_iters = float(np.mean(s[args.warmup:, :, 0])) if args.steps else 0.0
    lz = logz.cpu().numpy()
    del eng
    # the same restarts on the one-restart engine, one after another
    one = DeviceEM(sp, L, basis=B, scan=ScanConfig(warmup=args.warm_steps))
    one.adaptive = True
    one.set_transition(tr)
    W1 = torch.empty((NB, N), dtype=torch.float64, device=dev)
    mu1, nu1 = torch.zeros_like(W1), torch.zeros_like(W1)
    cnt1 = torch.zeros(1, dtype=torch.int64, device=dev)
    st1 = torch.zeros((n_all, 4), dtype=torch.float64, device=dev)
    lh1 = torch.zeros((n_all, adam.maxiter), dtype=torch.float64, device=dev)
    eh1 = torch.zeros_like(lh1)
    lz1 = torch.zeros(n_all, dtype=torch.float64, device=dev)
    seq = 0.0
    n_seq = min(R, 2)                      # time 2 restarts, scale to R
    for r in range(n_seq):
        def fresh1(r=r):
            one.set_log_posterior(lps[r])
            one.reset_adaptive()
            W1.copy_(torch.as_tensor(W0.astype(np.float64), device=dev))
            mu1.zero_(); nu1.zero_(); cnt1.zero_()

        def it1(i):
            one.m_step(W1, mu1, nu1, cnt1, adam, st1[i], lh1[i], eh1[i])
            one.compute_tuning(W1)
            one.e_step(1.0, lz1[i:i + 1])
        seq += run(fresh1, it1)
    seq_rate = world * n_seq * args.steps / seq
    value = world * R * args.steps / elapsed
    out = {
        "metric": f"restart EM iters/sec at {cfg.upper()} (N={N}, T={T}, L={L}), {R} restarts per GPU",
        "value": value,
        "unit": "restart EM iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 state / int8-exact emission / f64 stats",
        "data": "synthetic (spikes sampled from the model; seeds of BASELINE.md section 2)",
        "config": {"workload": f"{cfg}: {R} restarts x PoissonGPLVMJump1D.fit_em N={N} T={T} L={L} nb={NB} per "
                               f"GPU as one batched fit; one step = one EM iteration of every restart",
                   "n_neuron": N, "n_time": T, "n_latent_bin": L, "restarts_per_gpu": R,
                   "parallelism": f"restarts {R} x {world} GPUs"},
        "sequential_restart_iters_per_s": seq_rate,
        "batched_vs_sequential": value / seq_rate,
        "kernels_ms": {k: round(v[1], 4) for k, v in summ.items()},
        "kernel_calls": {k: v[0] for k, v in summ.items()},
        "adam_iters_mean": adam_iters,
        "chunk": max(32, -(-R * T // 2048)),
        "log_marginal_last": [float(v) for v in lz[n_all - 1]],
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` outside a launcher: run N ranks (one process per GPU) through
    torch.distributed.run on this node, rendezvous on 127.0.0.1.  The parent imports
    nothing GPU-related and only forwards the children's exit status; rank 0 prints the
    JSON line.  Under torchrun (WORLD_SIZE set) bench.py runs as one rank directly."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(n)}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.run(cmd, env=env).returncode
    if rc:
        sys.exit(rc)


def world_info():
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 without it)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def launcher_selftest(args):
    """The launcher's rank protocol on the CPU (gloo): every rank times the same host
    loop between two barriers, the max over ranks is taken with all_reduce(MAX), rank 0
    prints one JSON line whose n_gpus is the world size the process group saw."""
    import torch
    import torch.distributed as dist
    world, rank, _ = world_info()
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    x = np.random.default_rng(rank).random((256, 256))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = np.tanh(x @ x.T / 256.0)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    te = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "launcher selftest (host loop)", "value": world * args.steps / float(te[0]),
                          "unit": "loops/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ranks_max_s": float(te[0])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def decode_leg(y, tuning, L, reps=2):
    """decode_latent (core.py:454-497) at the bench shape with the fitted tuning: wall time
    of the public call (spikes uploaded, smoother, pairwise joint, every returned array
    copied to numpy; the first call loads code objects and is not counted), then the
    device sections of one decode under HIP events.  Default exact path (dense
    log-domain scans, f64 log-domain joint) and the banded path (decode_exact=False)."""
    import torch
    from poor_man_gplvm_amd import PoissonGPLVMJump1D, ScanConfig
    from poor_man_gplvm_amd.engine import KernelTimer
    out = {}
    for name, exact in (("exact", True), ("banded", False)):
        m = PoissonGPLVMJump1D(y.shape[1], n_latent_bin=L, tuning_lengthscale=10.0, movement_variance=1.0,
                               scan_config=ScanConfig(decode_exact=exact))
        m.decode_latent(y, tuning=tuning)
        walls = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = m.decode_latent(y, tuning=tuning)
            walls.append(time.perf_counter() - t0)
        eng = m._decode_engine(y, tuning, {}, None, None)
        eng.timer = KernelTimer()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m._decode_on(eng, {}, None, 1.0)
        torch.cuda.synchronize()
        dev_wall = time.perf_counter() - t0
        summ = eng.timer.summary()
        eng.timer = None
        sec = {k: round(v[0] * v[1], 3) for k, v in summ.items()}
        out[name] = {"wall_s": min(walls), "smoother_joint_call_s": dev_wall,
                     "device_ms": round(sum(sec.values()), 3), "sections_ms": sec,
                     "log_marginal_final": float(r["log_marginal_final"])}
        del m, eng, r
        torch.cuda.empty_cache()
    T = y.shape[0]
    jl = out["exact"]["sections_ms"].get("joint_log", 0.0)
    if jl > 0:
        terms = 4.0 * L * L * (T - 1)
        out["exact"]["joint_log_terms_per_s"] = terms / (jl * 1e-3)
    out["note"] = ("wall_s: public decode_latent, best of %d after one untimed call (upload of y, prepare, "
                   "scans, joint, host copies); sections_ms: HIP events of the smoother + joint of one decode; "
                   "joint_log_terms_per_s: 4 L^2 (T-1) log-domain terms / k_joint_log time" % reps)
    return out


def api_fit_wall(y, B, W0, lp0, L, n_iter=20):
    """Wall time of the public PoissonGPLVMJump1D.fit_em(n_iter=20) on the same data,
    end to end: host->device upload of y, 20 EM iterations, and the result dict
    (posterior (T,2,L), log posteriors, histories) copied back to numpy.  Cold: the
    process's first public fit (its page-locked result buffers are allocated and pinned
    on the way); warm: a second fit after the first result was dropped (the buffers come
    from the pinned-block cache)."""
    import gc
    import torch
    from poor_man_gplvm_amd import PoissonGPLVMJump1D

    def one():
        m = PoissonGPLVMJump1D(y.shape[1], n_latent_bin=L, tuning_lengthscale=10.0, movement_variance=1.0)
        m.tuning_basis = B
        m.params = W0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = m.fit_em(y, n_iter=n_iter, log_posterior_init=lp0)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, float(res["log_marginal"])

    cold, lm = one()
    gc.collect()
    warm, _ = one()
    return {"n_iter": n_iter, "wall_s": cold, "em_iters_per_s": n_iter / cold,
            "wall_s_warm": warm, "em_iters_per_s_warm": n_iter / warm, "log_marginal": lm,
            "note": "includes PCIe upload of y and the copy of every returned (T,2,L)/(T,L) array to host; "
                    "wall_s = cold (first public fit of the process), wall_s_warm = a second fit"}


if __name__ == "__main__":
    main()
