"""Time-sharded EM: one long spike train split into contiguous time shards, one per
rank (BASELINE config C4: T = 1e6 over 8 MI355X), or several virtual shards on one
device (the same algorithm, used by the single-GPU tests).

Reference: the chunk loop of decoder.smooth_all_step_combined_ma_chunk
(decoder.py:258-332) carries the filter state forward (post[-1], logZ, :283-304) and
the smoother state backward (acausal[0], :313-326) from chunk to chunk; the M-step's
sufficient statistics (fit_tuning_helper.get_statistics, :28-42) and the log marginal
(decoder.py:169) are sums over time.  Here the chunks of one shard live on one GPU
and the shards on different GPUs:

  M-step   y_w, t_w over the shard's own time range (pmg_suffstats*), then ONE
           all-reduce(SUM) of (y_w, t_w) in f64 over RCCL; the Adam loop
           (pmg_mstep_adam) then runs replicated on every rank -- it is deterministic
           and sees bit-identical statistics (an all-reduce leaves the same bits on
           every rank), so W stays identical without a broadcast.
  E-step   emission + chunk-parallel forward/backward on the shard EXTENDED by a halo
           of H steps on each side (H a multiple of the chunk), so that the shard's
           first own filter state and last own smoother state are already warmed up
           by the neighbour's data (HMM forgetting, as between chunks on one GPU).
           Then carry rounds: every rank sends its last own filter state to the right
           neighbour (its first own smoother state to the left one) over
           point-to-point send/recv; the receiver writes it into the boundary slot of
           its workspace (pmg_fwdbwd_state) and re-runs phase 2 of the scan, which
           verifies the boundary in the Hilbert metric and repairs the shard exactly
           as it repairs an interior chunk boundary.  Rounds repeat until no rank
           repaired anything (all-reduce MAX of a flag): exactness propagates one
           shard per round from rank 0 (exact start) and rank R-1 (exact end), so at
           most R-1 rounds are ever needed; converged halos need one.
           logZ = all-reduce(SUM) of the shard's own sum_t logc_t.

Communication per EM iteration: 1 all-reduce of L*(N+1) f64 (8.4 MB at C4), plus
per carry round one 2*Lpad f32 send/recv each way and a 4-byte all-reduce.  All of
it is latency-bound on xGMI.
"""
from __future__ import annotations

import ctypes
import math
import time
from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .engine import AdamConfig, DeviceEM, ScanConfig, SpikeData, _ru


# --------------------------------------------------------------------------- layout
@dataclass(frozen=True)
class ShardLayout:
    """Own range [start, stop) and extended range [ext_start, ext_stop) of one shard;
    chunk boundaries of the extended range coincide with the global chunk grid."""
    rank: int
    world: int
    start: int
    stop: int
    ext_start: int
    ext_stop: int
    chunk: int

    @property
    def T_own(self):
        return self.stop - self.start

    @property
    def T_ext(self):
        return self.ext_stop - self.ext_start

    @property
    def left(self):           # halo steps before the own range
        return self.start - self.ext_start

    @property
    def right(self):          # halo steps after the own range
        return self.ext_stop - self.stop

    @property
    def n_chunks(self):       # chunks of the extended range
        return (self.T_ext + self.chunk - 1) // self.chunk

    @property
    def c_first(self):        # first own chunk (local index)
        return self.left // self.chunk

    @property
    def c_last(self):         # last own chunk (local index)
        return (self.left + self.T_own + self.chunk - 1) // self.chunk - 1


def shard_layout(T: int, world: int, chunk: int | None = None, halo: int = 512,
                 scan: ScanConfig | None = None, dense: bool = False) -> list[ShardLayout]:
    """Split [0, T) into `world` contiguous shards of whole chunks (the last shard takes
    the remainder), each extended by `halo` steps (rounded up to whole chunks) on the
    sides that have a neighbour.  dense: the default chunk of the dense log-domain scans
    (custom / wide continuous kernels)."""
    if world < 1 or T < 1:
        raise ValueError("need T >= 1 and world >= 1")
    scan = scan or ScanConfig()
    Tw = int(math.ceil(T / world))
    C = int(chunk) if chunk else (scan.chunk_dense_for(Tw) if dense else scan.chunk_for(Tw))
    n_chunks = (T + C - 1) // C
    if n_chunks < world:
        raise ValueError(f"T={T} gives {n_chunks} chunks of {C}: fewer than {world} shards")
    H = _ru(max(int(halo), 1), C)
    base, rem = divmod(n_chunks, world)
    out, c0 = [], 0
    for r in range(world):
        nc = base + (1 if r < rem else 0)
        s, e = c0 * C, min((c0 + nc) * C, T)
        c0 += nc
        a = max(0, s - H) if r > 0 else 0
        b = min(T, e + H) if r < world - 1 else T
        out.append(ShardLayout(r, world, s, e, a, b, C))
    assert out[-1].stop == T
    return out


# --------------------------------------------------------------------------- comms
class LocalComm:
    """All shards in this process (virtual ranks on one device), in rank order."""

    def __init__(self, world: int):
        self.world = world
        self.ranks = list(range(world))

    def allreduce_sum(self, per_shard):
        """per_shard[i] = tensors of local shard i; sums over shards in rank order and
        leaves the same bits in every shard."""
        for k in range(len(per_shard[0])):
            acc = per_shard[0][k].clone()
            for i in range(1, len(per_shard)):
                acc += per_shard[i][k]
            for i in range(len(per_shard)):
                per_shard[i][k].copy_(acc)

    def allreduce_max_int(self, vals):
        return max(int(v) for v in vals)

    def shift(self, send, recv, direction):
        """direction +1: shard r's send -> shard r+1's recv; -1: r -> r-1.  Entries are
        None where there is no neighbour."""
        for i, r in enumerate(self.ranks):
            dst = r + direction
            if 0 <= dst < self.world and send[i] is not None:
                recv[self.ranks.index(dst)].copy_(send[i])

    def gather_rank0(self, parts):
        return [p.cpu() for p in parts]

    def allreduce_process_sum(self, x):
        """x is already summed over this process's shards, i.e. over all ranks."""
        return np.asarray(x, np.float64)

    def allreduce_np(self, per_shard):
        """Sum of host arrays over shards (rank order); the same array for every shard."""
        acc = np.array(per_shard[0], dtype=np.float64, copy=True)
        for a in per_shard[1:]:
            acc = acc + a
        return acc

    def allgather_cols(self, slices, fulls, bounds):
        """slices[i]: (rows, b-a) device tensor of local shard i (neuron block
        bounds[rank]); every full (rows, N) tensor receives every block."""
        for i, r in enumerate(self.ranks):
            a, b = bounds[r]
            for f in fulls:
                f[:, a:b].copy_(slices[i])


class DistComm:
    """One shard per process over torch.distributed: backend "nccl" (= RCCL over xGMI
    on ROCm) with device tensors, or "gloo" with host staging."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.ranks = [self.rank]
        self.host = dist.get_backend(group) == "gloo"

    def _stage(self, t):
        return t.cpu() if (self.host and t.is_cuda) else t

    def allreduce_sum(self, per_shard):
        (ts,) = per_shard
        for t in ts:
            s = self._stage(t)
            self.dist.all_reduce(s, op=self.dist.ReduceOp.SUM, group=self.group)
            if s is not t:
                t.copy_(s)

    def allreduce_max_int(self, vals):
        dev = torch.device("cpu") if self.host else torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([int(max(vals))], dtype=torch.int64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def shift(self, send, recv, direction):
        (snd,), (rcv,) = send, recv
        dst, src = self.rank + direction, self.rank - direction
        ops, staged = [], None
        if 0 <= dst < self.world and snd is not None:
            ops.append(self.dist.P2POp(self.dist.isend, self._stage(snd).contiguous(), dst, self.group))
        if 0 <= src < self.world and rcv is not None:
            staged = self._stage(rcv)
            ops.append(self.dist.P2POp(self.dist.irecv, staged, src, self.group))
        if ops:
            for w in self.dist.batch_isend_irecv(ops):
                w.wait()
        if staged is not None and staged is not rcv:
            rcv.copy_(staged)

    def allreduce_process_sum(self, x):
        return self.allreduce_np([x])

    def allreduce_np(self, per_shard):
        (a,) = per_shard
        dev = torch.device("cpu") if self.host else torch.device("cuda", torch.cuda.current_device())
        t = torch.as_tensor(np.asarray(a, np.float64), device=dev).contiguous()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy()

    def allgather_cols(self, slices, fulls, bounds):
        (mine,) = slices
        wmax = max(b - a for a, b in bounds)
        buf = torch.zeros((mine.shape[0], wmax), dtype=mine.dtype, device=mine.device)
        buf[:, :mine.shape[1]].copy_(mine)
        src = self._stage(buf)
        parts = [torch.empty_like(src) for _ in range(self.world)]
        self.dist.all_gather(parts, src, group=self.group)
        for r, (a, b) in enumerate(bounds):
            blk = parts[r][:, :b - a].to(mine.device)
            for f in fulls:
                f[:, a:b].copy_(blk)

    def gather_rank0(self, parts):
        """Variable-length slices to rank 0 (host tensors there; [] elsewhere)."""
        (mine,) = parts
        if self.world == 1:
            return [mine.cpu()]
        shapes = [None] * self.world
        self.dist.all_gather_object(shapes, tuple(mine.shape), group=self.group)
        if self.rank == 0:
            out = [mine.cpu()]
            for r in range(1, self.world):
                buf = torch.empty(shapes[r], dtype=mine.dtype,
                                  device="cpu" if (self.host or not mine.is_cuda) else mine.device)
                self.dist.recv(buf, src=r, group=self.group)
                out.append(buf.cpu())
            return out
        self.dist.send(self._stage(mine.contiguous()), dst=0, group=self.group)
        return []


# --------------------------------------------------------------------------- Adam
def neuron_bounds(N: int, world: int):
    """Contiguous neuron blocks of the neuron-sharded M-step, one per rank."""
    edges = [round(r * N / world) for r in range(world + 1)]
    return [(edges[r], edges[r + 1]) for r in range(world)]


def adam_stop_body(losses, j0, maxiter, tol, state):
    """The while-loop rule of fit_tuning_helper.make_adam_runner.run (:154-164) over the
    global losses of bodies j0, j0+1, ... (losses[i] is computed at W_{j0+i}, before that
    body's update).  state carries loss_prev across calls.  Returns the body after whose
    update the loop stops, or None if it runs past these bodies.  The same rule as the
    persistent kernel's decision pipeline (mstep_adam.hip)."""
    for i, loss in enumerate(losses):
        j = j0 + i
        loss = float(loss)
        if j == 0:
            state['prev'] = loss
        rel = abs(loss - state['prev']) / max(abs(loss), 1e-8)
        cont = (j + 1 < maxiter - 1) and ((j + 1 < 5) or (rel > tol))
        state['prev'] = loss
        if not cont:
            return j
    return None


SPEC_BATCH = 16     # bodies per speculative launch of the neuron-sharded Adam (the exact-F refresh period)


def speculative_adam(run, snapshot, restore, allreduce, maxiter, tol, batch=SPEC_BATCH, max_batch=None):
    """Neuron-sharded Adam loop with the reference's global stop rule.

    Every rank runs its own neuron slice (the loss and the gradient norm are sums over
    neurons plus per-weight prior terms), `batch` bodies per launch with tol < 0 (no local stop), then
    ONE all-reduce of the batch's per-body loss / squared-gradient partials decides on
    the global sums, in the same order on every rank.  A stop inside the batch restores
    the batch-start snapshot and re-runs the bodies up to the stopping one, so every rank
    ends with exactly the state the unsharded loop reaches (batch = 16 keeps the
    persistent kernel's exact-F refresh, every 16 bodies, on the same bodies).

      run(kmax) -> list over local slices of (n_iter, loss_hist, err_hist) host arrays
                   (the kernel's outputs for maxiter = kmax, tol < 0)
      snapshot() / restore(): all local slices' (W, mu, nu, count)
      allreduce(x) -> sum over ranks of the local sum x (host float64 arrays)
    max_batch: the launches double from `batch` up to max_batch bodies (multiples of
    `batch`, so every launch still starts on a refresh body): fewer host round trips for
    long loops, at the price of up to max_batch - 1 speculative bodies past the stop.
    Returns dict(n_iter, final_loss, final_error, loss_history, error_history, loss0)."""
    if maxiter <= 1:   # eval only: the loss at W_0, no update
        outs = run(1)
        loc = np.array([[o[1][0] for o in outs], [o[2][0] ** 2 for o in outs]]).sum(axis=1)
        g = allreduce(loc)
        return dict(n_iter=1, final_loss=float(g[0]), final_error=float(np.sqrt(g[1])),
                    loss_history=np.array([g[0]]), error_history=np.array([np.sqrt(g[1])]), loss0=float(g[0]))
    mb = batch if max_batch is None else max(batch, (int(max_batch) // batch) * batch)
    j0, st = 0, {}
    lh, eh = [], []
    cur = batch
    while True:
        snap = snapshot()
        outs = run(cur + 1)
        nb = int(outs[0][0]) - 1                        # bodies this launch ran: exactly `cur` (tol < 0)
        if any(int(o[0]) - 1 != nb for o in outs):
            raise RuntimeError("speculative_adam: local slices ran different body counts")
        loc = np.zeros((2, nb))
        for n_iter, lhist, ehist in outs:
            loc[0] += np.asarray(lhist[1:nb + 1], np.float64)
            loc[1] += np.asarray(ehist[1:nb + 1], np.float64) ** 2
        g = allreduce(loc)
        losses, errs = g[0], np.sqrt(g[1])
        j = adam_stop_body(losses, j0, maxiter, tol, st)
        stop_at = nb - 1 if j is None else j - j0
        lh.extend(losses[:stop_at + 1])
        eh.extend(errs[:stop_at + 1])
        if j is not None:
            if stop_at < nb - 1:       # the stop lies inside the batch: replay up to it
                restore(snap)
                run(stop_at + 2)
            hist_l = np.array([lh[0]] + lh)
            hist_e = np.array([eh[0]] + eh)
            return dict(n_iter=j + 2, final_loss=float(lh[-1]), final_error=float(eh[-1]),
                        loss_history=hist_l, error_history=hist_e, loss0=float(lh[0]))
        j0 += nb
        cur = min(2 * cur, mb)


# --------------------------------------------------------------------------- shard
class ShardEM(DeviceEM):
    """DeviceEM over one shard's extended range, with own-range statistics and the
    boundary-state views the carry rounds exchange."""

    PLANES = False      # the shard's statistics run over its own rows of the f32 P

    def __init__(self, lay: ShardLayout, y, L, basis, scan: ScanConfig, ma_neuron=None, device=None):
        self.lay = lay
        y_ext = np.asarray(y[lay.ext_start:lay.ext_stop])
        ma = None
        if ma_neuron is not None:
            ma = np.asarray(ma_neuron, np.float32)
            if ma.ndim == 2:
                ma = ma[lay.ext_start:lay.ext_stop]
        sp = SpikeData(y_ext, ma, device=device)
        # one chunk grid for both passes: the carry slots sit on the shard's chunk boundaries
        sc = ScanConfig(chunk=lay.chunk, warmup=scan.warmup, tol=scan.tol, adaptive=scan.adaptive,
                        max_warmup=scan.max_warmup, min_warmup=scan.min_warmup, chunk_bwd=lay.chunk)
        super().__init__(sp, L, basis=basis, scan=sc)
        assert self.C == lay.chunk and self.Cb == lay.chunk
        self.Lpad = int(self.lib.pmg_fwdbwd_lpad(self.L))
        To, hl = lay.T_own, lay.left
        self.own = slice(hl, hl + To)
        self.ybt_own = None
        if sp.ybt is not None:
            self.Tp_own = _ru(To, 64)
            self.ybt_own = torch.empty((sp.Np, self.Tp_own), dtype=torch.int16, device=self.dev)
            nat.check(self.lib.pmg_spikes_bf16t(nat.ptr(sp.yext[self.own]), To, sp.Np, nat.ptr(self.ybt_own),
                                                self.Tp_own, nat.stream_handle()), "pmg_spikes_bf16t")

    def state(self, which: int, c: int) -> torch.Tensor:
        """(2*Lpad,) f32 view of a boundary slot inside the scan workspace (the dense
        log-domain scans: (2*Lp,) f64 log state, pmg_dense_state)."""
        if self.dense:
            p = self.lib.pmg_dense_state(nat.ptr(self.ws_dense), self.T, self.L, self.Cd, int(which), int(c))
            if not p:
                raise nat.NativeError(f"pmg_dense_state({which}, {c}) failed")
            off = int(p) - self.ws_dense.data_ptr()
            lp = int(self.lib.pmg_dense_lpad(self.L))
            return self.ws_dense[off:off + 16 * lp].view(torch.float64)
        p = self.lib.pmg_fwdbwd_state(nat.ptr(self.ws_fb), self.T, self.L, self.C, int(which), int(c))
        if not p:
            raise nat.NativeError(f"pmg_fwdbwd_state({which}, {c}) failed")
        off = int(p) - self.ws_fb.data_ptr()
        return self.ws_fb[off:off + 8 * self.Lpad].view(torch.float32)

    def suffstats_own(self):
        lay, sh = self.lay, nat.stream_handle()
        P = self.P[self.own]
        with self._t('suffstats'):
            if self.ybt_own is not None:
                nat.check(self.lib.pmg_suffstats_bf16(nat.ptr(P), nat.ptr(self.ybt_own), lay.T_own, self.Tp_own,
                                                      self.L, self.N, self.sp.Np, nat.ptr(self.yw),
                                                      nat.ptr(self.tw), nat.ptr(self.ws_ss), self.ws_ss.numel(),
                                                      sh), "pmg_suffstats_bf16")
            else:
                nat.check(self.lib.pmg_suffstats(nat.ptr(P), nat.ptr(self.sp.yext[self.own]), lay.T_own, self.L,
                                                 self.N, self.sp.Np, nat.ptr(self.yw), nat.ptr(self.tw),
                                                 nat.ptr(self.ws_ss), self.ws_ss.numel(), sh), "pmg_suffstats")

    def forward_phase2(self, likelihood_scale, logz_scratch):
        if self.dense:
            with self._t('forward_carry'):
                nat.check(self.lib.pmg_dense_forward_phase(
                    nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.ll64), nat.ptr(self.mref), self.T,
                    ctypes.byref(self._tr_d), float(likelihood_scale), self.Cd, int(self.warm[0]),
                    float(self.scan.tol), nat.ptr(self.alpha), nat.ptr(self.log_alpha), nat.ptr(self.logc),
                    nat.ptr(logz_scratch), nat.ptr(self.ws_dense), self.ws_dense.numel(), nat.stream_handle(), 2),
                    "pmg_dense_forward_phase")
            return
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.mref), self.T, ctypes.byref(self._tr_c),
                float(likelihood_scale), self.C, int(self.warm[0]), float(self.scan.tol), nat.ptr(self.alpha),
                nat.ptr(self.logc), nat.ptr(logz_scratch), nat.ptr(self.ws_fb), self.ws_fb.numel(),
                nat.stream_handle())
        with self._t('forward_carry'):
            nat.check(self.lib.pmg_forward_filter_phase(*args, 2 | self.alpha_bits | self._seg_bits()),
                      "pmg_forward_filter")

    def backward_phase2(self, likelihood_scale, P=True, gamma=None):
        if self.dense:
            with self._t('backward_carry'):
                nat.check(self.lib.pmg_dense_backward_phase(
                    nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.ll64), nat.ptr(self.log_alpha), self.T,
                    ctypes.byref(self._tr_d), float(likelihood_scale), self.Cd, int(self.warm[1]),
                    float(self.scan.tol), nat.ptr(self._P) if P else None, nat.ptr(gamma), None, None, None,
                    nat.ptr(self.ws_dense), self.ws_dense.numel(), nat.stream_handle(), 2),
                    "pmg_dense_backward_phase")
            return
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.alpha), self.T, ctypes.byref(self._tr_c),
                float(likelihood_scale), self.C, int(self.warm[1]), float(self.scan.tol),
                nat.ptr(self.P) if P else None, nat.ptr(gamma), None, nat.ptr(self.ws_fb),
                self.ws_fb.numel(), nat.stream_handle())
        with self._t('backward_carry'):
            nat.check(self.lib.pmg_backward_smoother_phase(*args, 2 | self._seg_bits()), "pmg_backward_smoother")

    def repair_count(self):
        """(forward, backward) chunk-recompute counters (device tensor)."""
        w = self.ctl_words()
        return torch.stack([w[nat.CTL_FWD + nat.CTL_REPAIRS], w[nat.CTL_BWD + nat.CTL_REPAIRS]])

    def own_logz(self, out):
        torch.sum(self.logc[self.own], dim=0, keepdim=True, out=out)


class TimeShardedEM:
    """The EM loop of core.py:650-676 over time shards (see the module docstring)."""

    def __init__(self, y, basis, transition, comm, layouts, scan: ScanConfig | None = None,
                 ma_neuron=None, ma_latent=None, device=None, neuron_sharded=False):
        self.comm = comm
        self.lays = [layouts[r] for r in comm.ranks]
        self.world = comm.world
        B = np.asarray(basis, np.float32)
        self.L = B.shape[0]
        scan = scan or ScanConfig()
        self.shards = [ShardEM(lay, y, self.L, B, scan, ma_neuron, device) for lay in self.lays]
        for s in self.shards:
            s.adaptive = True       # one fit: adaptive warm-up across its E-steps
            s.set_transition(transition)
            s.set_ma_latent(ma_latent)
        self.dev = self.shards[0].dev
        self.carry_rounds = [0, 0]     # carry rounds of the last E-step (forward, backward)
        # neuron-sharded Adam (one neuron block per rank) instead of the replicated loop
        self.neuron_sharded = bool(neuron_sharded) and self.world > 1
        self._slices = None

    def set_timer(self, timer):
        for s in self.shards:
            s.timer = timer

    def _carry(self, kind, likelihood_scale, scratch, gamma=None):
        """kind 0: filter state to the right neighbour, 1: beta to the left neighbour."""
        if self.world == 1:
            return 0
        last = self.world - 1
        gamma = gamma or [None] * len(self.shards)
        rounds = 0
        while True:
            send, recv = [], []
            for s in self.shards:
                lay = s.lay
                if kind == 0:
                    send.append(s.state(nat.STATE_FWD_OUT, lay.c_last).clone() if lay.rank < last else None)
                    recv.append(s.state(nat.STATE_FWD_OUT, lay.c_first - 1) if lay.rank > 0 else None)
                else:
                    send.append(s.state(nat.STATE_BWD_FIRST, lay.c_first).clone() if lay.rank > 0 else None)
                    recv.append(s.state(nat.STATE_BWD_FIRST, lay.c_last + 1) if lay.rank < last else None)
            before = [s.repair_count() for s in self.shards]
            self.comm.shift(send, recv, +1 if kind == 0 else -1)
            for s, g in zip(self.shards, gamma):
                if kind == 0:
                    s.forward_phase2(likelihood_scale, scratch)
                else:
                    s.backward_phase2(likelihood_scale, True, g)
            rounds += 1
            changed = [int(s.repair_count()[kind].item() > b[kind].item()) for s, b in zip(self.shards, before)]
            # exactness moves at least one shard per round: R rounds always suffice
            if self.comm.allreduce_max_int(changed) == 0 or rounds >= self.world:
                return rounds

    def e_step(self, likelihood_scale, logz_out, gamma=None):
        """logz_out: (1,) f64 device tensor <- the global log marginal (decoder.py:169)."""
        if getattr(self, '_estep_bufs', None) is None:     # scratch and per-shard logZ parts, once
            self._estep_bufs = (torch.empty(1, dtype=torch.float64, device=self.dev),
                                [torch.empty(1, dtype=torch.float64, device=self.dev) for _ in self.shards])
        scratch, lzp = self._estep_bufs
        for s in self.shards:
            s.emission(likelihood_scale)
            s.forward(likelihood_scale, scratch, keep_alpha=gamma is not None)
        self.carry_rounds[0] = self._carry(0, likelihood_scale, scratch)
        parts = []
        for s, buf in zip(self.shards, lzp):
            parts.append([buf])
            s.own_logz(buf)
        for s, g in zip(self.shards, gamma or [None] * len(self.shards)):
            s.backward(likelihood_scale, True, g)
        self.carry_rounds[1] = self._carry(1, likelihood_scale, scratch, gamma)
        for s in self.shards:
            s._snapshot_repairs()
        self.comm.allreduce_sum(parts)
        logz_out.copy_(parts[0][0])

    def m_step(self, Ws, mus, nus, cnts, cfg: AdamConfig, stats, lh, eh):
        for s in self.shards:
            s.suffstats_own()
        self.comm.allreduce_sum([[s.yw, s.tw] for s in self.shards])
        if self.neuron_sharded:
            self._adam_neuron_sharded(Ws, mus, nus, cnts, cfg, stats, lh, eh)
        else:
            for s, W, mu, nu, c in zip(self.shards, Ws, mus, nus, cnts):
                s.adam(W, mu, nu, c, cfg, stats, lh, eh)
        for s, W in zip(self.shards, Ws):
            s.compute_tuning(W)

    def _adam_neuron_sharded(self, Ws, mus, nus, cnts, cfg: AdamConfig, stats, lh, eh):
        """Rank r runs Adam on neuron block bounds[r] only (speculative_adam); W is then
        all-gathered so every rank holds the full W for the tuning.  mu / nu of a block
        live on its rank only (the unused columns of mus / nus are not maintained)."""
        N = Ws[0].shape[1]
        bounds = neuron_bounds(N, self.world)
        if self._slices is None:
            self._slices = []
            for s, r, mu, nu in zip(self.shards, self.comm.ranks, mus, nus):
                a, b = bounds[r]
                self._slices.append({'mu': mu[:, a:b].contiguous(), 'nu': nu[:, a:b].contiguous()})
        sl = []
        for s, r, W, c, d in zip(self.shards, self.comm.ranks, Ws, cnts, self._slices):
            a, b = bounds[r]
            d['W'] = W[:, a:b].contiguous()
            d['yw'] = s.yw[:, a:b].contiguous()
            d['count'] = c
            sl.append(d)
        mi = max(int(cfg.maxiter), 1)
        ns = len(self.shards)
        # per local slice: stats (4) | loss history | error history (hl entries each: a
        # speculative launch writes SPEC_BATCH + 1 of them whatever maxiter is), so that one
        # launch per slice and ONE device-to-host copy serve a batch (no host sync between
        # the slices)
        hl = max(mi, SPEC_BATCH + 1) + 1
        hist = torch.zeros((ns, 4 + 2 * hl), dtype=torch.float64, device=self.dev)

        def run(kmax):
            # tol < 0: the local stop rule (rel > tol) never fires, so every rank runs exactly
            # kmax - 1 bodies (a repeated partial loss, rel == 0, would stop a tol = 0 loop
            # early on one rank only and desynchronise the loss all-reduce)
            c = AdamConfig(lr=cfg.lr, maxiter=kmax, tol=-1.0, prior_std=cfg.prior_std, b1=cfg.b1, b2=cfg.b2,
                           eps=cfg.eps, eps_root=cfg.eps_root)
            k = int(kmax)
            if k > hl:
                raise ValueError(f"speculative Adam launch of {k} bodies > history slots {hl}")
            for i, (s, d) in enumerate(zip(self.shards, sl)):
                h = hist[i]
                s.adam(d['W'], d['mu'], d['nu'], d['count'], c, h[:4], h[4:4 + hl], h[4 + hl:], yw=d['yw'])
            sel = torch.cat([hist[:, :1], hist[:, 4:4 + k], hist[:, 4 + hl:4 + hl + k]], dim=1).cpu().numpy()
            outs = []
            for row in sel:
                n = int(row[0])
                outs.append((n, row[1:1 + n], row[1 + k:1 + k + n]))
            return outs

        def snapshot():
            return [(d['W'].clone(), d['mu'].clone(), d['nu'].clone(), d['count'].clone()) for d in sl]

        def restore(snap):
            for d, (W, mu, nu, c) in zip(sl, snap):
                d['W'].copy_(W)
                d['mu'].copy_(mu)
                d['nu'].copy_(nu)
                d['count'].copy_(c)

        res = speculative_adam(run, snapshot, restore, self.comm.allreduce_process_sum, int(cfg.maxiter),
                               float(cfg.tol), batch=SPEC_BATCH)
        self.comm.allgather_cols([d['W'] for d in sl], Ws, bounds)
        n = res['n_iter']
        stats.copy_(torch.tensor([n, res['final_loss'], res['final_error'], res['loss0']], dtype=torch.float64))
        k = min(n, lh.shape[0])
        lh[:k].copy_(torch.as_tensor(res['loss_history'][:k]))
        eh[:k].copy_(torch.as_tensor(res['error_history'][:k]))


def run_em_timesharded(y, params, basis, log_posterior_init, n_iter, transition, comm=None, world=None,
                       ma_neuron=None, ma_latent=None, likelihood_scale=1.0, adam: AdamConfig | None = None,
                       scan: ScanConfig | None = None, halo=512, chunk=None, timing=None, gather=True,
                       timer=None, neuron_sharded=False):
    """Time-sharded counterpart of core.run_em.  `comm`: DistComm (one shard per
    rank), or None for `world` virtual shards on this device (LocalComm).  Returns
    (res, info); res has run_em's per-fit keys with the per-time outputs concatenated
    over shards.  With DistComm and `gather` they are gathered on rank 0 and the other
    ranks get res=None; without `gather` every rank returns its own slice.
    neuron_sharded: each rank runs the Adam M-step on its own neuron block
    (speculative_adam) instead of the whole replicated loop."""
    adam = adam or AdamConfig()
    if comm is None:
        comm = LocalComm(int(world or 1))
    if not hasattr(y, "shape"):
        y = np.asarray(y)
    T = int(y.shape[0])
    from .gp_kernel import DenseTransition
    lays = shard_layout(T, comm.world, chunk=chunk, halo=halo, scan=scan,
                        dense=isinstance(transition, DenseTransition))
    eng = TimeShardedEM(y, basis, transition, comm, lays, scan, ma_neuron, ma_latent,
                        neuron_sharded=neuron_sharded)
    if timer is not None:
        eng.set_timer(timer)
    dev = eng.dev
    for s in eng.shards:
        s.set_log_posterior(np.asarray(log_posterior_init[s.lay.ext_start:s.lay.ext_stop]))
    n = len(eng.shards)
    W0 = np.asarray(params, np.float64)
    Ws = [torch.as_tensor(W0, device=dev).contiguous() for _ in range(n)]
    mus = [torch.zeros_like(Ws[0]) for _ in range(n)]
    nus = [torch.zeros_like(Ws[0]) for _ in range(n)]
    cnts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(n)]
    mi = max(int(adam.maxiter), 1)
    stats = torch.zeros((n_iter, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_iter, mi), dtype=torch.float64, device=dev)
    eh = torch.zeros((n_iter, mi), dtype=torch.float64, device=dev)
    logz = torch.zeros(max(n_iter, 1), dtype=torch.float64, device=dev)
    gam = [torch.empty((s.T, 2, eng.L), dtype=torch.float32, device=dev) for s in eng.shards]
    rounds = []
    for i in range(n_iter):
        t0 = time.perf_counter()
        eng.m_step(Ws, mus, nus, cnts, adam, stats[i], lh[i], eh[i])
        eng.e_step(likelihood_scale, logz[i:i + 1], gamma=gam if i == n_iter - 1 else None)
        rounds.append(tuple(eng.carry_rounds))
        if timing is not None:
            torch.cuda.synchronize()
            timing.append(time.perf_counter() - t0)
    own = [g[s.own] for s, g in zip(eng.shards, gam)]
    parts = comm.gather_rank0(own) if gather else [o.cpu() for o in own]
    s_ = stats.cpu().numpy()
    lhn, ehn, lz = lh.cpu().numpy(), eh.cpu().numpy(), logz.cpu().numpy()
    for s in eng.shards:            # sticky device errors of every shard's calls
        s.emission_status()
        s.adam_status()
    info = {'layouts': lays, 'carry_rounds': rounds, 'params64': Ws[0].cpu().numpy(),
            'repairs': [s.repairs() for s in eng.shards], 'chunk': lays[0].chunk,
            'warmup': [list(s.warm) for s in eng.shards]}
    if not parts:
        return None, info
    posterior = torch.cat(parts, 0).numpy()
    m_step_res_l = {'n_iter': [], 'final_loss': [], 'final_error': [], 'loss_history': [], 'error_history': []}
    for i in range(n_iter):
        k = int(s_[i, 0])
        m_step_res_l['n_iter'].append(k)
        m_step_res_l['final_loss'].append(float(s_[i, 1]))
        m_step_res_l['final_error'].append(float(s_[i, 2]))
        m_step_res_l['loss_history'].append(lhn[i, :k].copy())
        m_step_res_l['error_history'].append(ehn[i, :k].copy())
    from .core import _masked_log
    mlat = None if ma_latent is None else np.asarray(ma_latent).astype(bool)
    with np.errstate(divide="ignore"):
        lpf = _masked_log(np.log(posterior), mlat)
    res = {'params': Ws[0].cpu().numpy().astype(np.float32),
           'tuning': eng.shards[0].tuning32.cpu().numpy(),
           'log_posterior_final': lpf,
           'log_marginal': float(lz[n_iter - 1]) if n_iter else float('nan'),
           'log_marginal_l': [float(v) for v in lz[:n_iter]],
           'posterior': posterior,
           'posterior_latent_marg': posterior.sum(axis=1),
           'posterior_dynamics_marg': posterior.sum(axis=2),
           'm_step_res_l': m_step_res_l}
    return res, info
