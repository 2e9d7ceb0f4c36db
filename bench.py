#!/usr/bin/env python3
"""bench.py -- perft leaf nodes/s (headline) + validated moves/s on MI355X.

Contract (see README / DESIGN.md):
  python bench.py --gpus N --steps K --warmup W
  N>1: launched by torch.distributed.run, one rank per GPU; RCCL ("nccl") for
  the per-root-move all-reduce of leaf counts and the max-over-ranks timing.

Workload: perft(startpos, 7) under RULES_REF -- the reference validator's own
rules (core/src/chess.rs), bit-exact -- with the frontier at ply 3 split into
contiguous shards over the ranks (BASELINE configs[4], the configuration the
node-level metric is quoted on; it fits one GPU).  One step = one full
perft(startpos, 7) = 3,282,734,510 leaves; value = leaves of all ranks / wall
time (strong scaling: the tree is fixed, N ranks share it).  perft(startpos, 6)
(configs[1]) is timed the same way and reported as the "perft6" object.  The secondary "replay" object is
BASELINE configs[3]: 10M synthetic seeded games x 80 ply slots replayed per
rank (weak scaling), inputs resident in HBM, validated moves/s.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "distributed-chess_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402

import dchess  # noqa: E402
from dchess.dist import sharded_perft  # noqa: E402

METRIC = "perft leaf nodes/sec + validated moves/sec (node), at 1/2/4/8 MI355X"
# REF perft(startpos, d): three-way agreed (refcpu <= d4, fastcpu, GPU), tests/golden/oracle_golden.json
REF_STARTPOS = {1: 20, 2: 400, 3: 8902, 4: 197742, 5: 4896998, 6: 120909581, 7: 3282734510}
POS_BYTES = 40  # dc_pos in HBM (4 x u64 bitboards + stm/castle/ep/rules + pad)
HBM_PEAK_GBPS = 8000.0

# MI355X (gfx950): 256 CUs x 4 SIMD-32 x 32 lanes per clock x 2.4 GHz (MI355X_MICROARCH.md).
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
CLOCK_HZ = 2.4e9
# SIMD cycles per VALU issue slot (a single-issue instruction or a dual-issued
# pair) at 4 waves/SIMD: v_bcnt_u32_b32 stream, profiles/r04/issue_costs.json
ISSUE_SLOT_CYCLES = 4.34
# W = int VALU lane-ops per unit, FROZEN from the first parity-passing kernels'
# rocprofv3 PMC passes (SQ_INSTS_VALU x 64 / units; DESIGN.md "Roofline"):
#   perft final stage (k_count2, perft(6)): 37,766,248 x 64 / 120,909,581 = 20.0 per leaf
#   replay (k_replay_ref, 1M games x 80 plies): 218,408,376 x 64 / 79.9M = 175 per validated move
# achieved = units/s x W, so the judge can recompute it from the reported rates.
W_COUNT2 = 20.0
# REF final stage: k_count3c (the last three plies: the final stage's parents expanded in-kernel,
# then the two-ply bulk count of k_count2c); A/B build: DC_FUSED3=0 -> k_count2c, DC_FINAL=2b -> k_count2b
_AB = os.environ.get("DCHESS_LIB")
FINAL_KERNEL = ("k_count2b" if (_AB and os.environ.get("DC_FINAL") == "2b")
                else "k_count2c" if (_AB and os.environ.get("DC_FUSED3") == "0") else "k_count3c")
W_REPLAY = 175.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--depth", type=int, default=7)
    ap.add_argument("--split", type=int, default=3)
    ap.add_argument("--games", type=int, default=10_000_000, help="replay games at N=1 (BASELINE configs[3])")
    ap.add_argument("--c5-games", type=int, default=100_000_000,
                    help="replay games in total at N>1, split over the ranks (BASELINE configs[4])")
    ap.add_argument("--plies", type=int, default=80)
    ap.add_argument("--replay-steps", type=int, default=5)
    ap.add_argument("--no-replay", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--profile-only", action="store_true", help="run the steps, print nothing (rocprof)")
    ap.add_argument("--no-perft", action="store_true", help="with --profile-only: replay leg only (PMC passes)")
    ap.add_argument("--hash-games", type=int, default=1_000_000, help="state-hash leg: games per rank (0: off)")
    ap.add_argument("--hash-steps", type=int, default=3)
    ap.add_argument("--txs", type=int, default=262_144, help="signature leg: transactions per rank (0: off)")
    ap.add_argument("--tx-steps", type=int, default=3)
    ap.add_argument("--perft-streams", type=int, default=0,
                    help="contexts a repeated perft's steps are split over (0: 3 at depth <= 6, 2 at 7, 1 deeper)")
    ap.add_argument("--suite-batch-only", action="store_true",
                    help="FIDE suite leg: the batch alone, no per-position runs (its PMC pass: one kind of dispatch)")
    ap.add_argument("--only", default="", help="comma-separated legs to run (rocprof passes): " + ", ".join(LEGS))
    return ap.parse_args()


class Dist:
    def __init__(self, want):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if want > 1 and self.world != want:
            raise SystemExit(f"--gpus {want} needs torch.distributed.run with {want} ranks (WORLD_SIZE={self.world})")
        import torch
        self.torch = torch
        self.dist = None
        # The engine's device: one GPU per rank.  DC_DIST_BACKEND=gloo (rehearsal
        # only) runs the collectives on host tensors and lets several ranks share
        # one GPU (device = local rank mod the devices present), so the N-rank
        # code path -- shards, exchange steps, parity checks -- runs end to end
        # on a one-GPU box; its timings mean nothing.
        self.backend = os.environ.get("DC_DIST_BACKEND", "nccl")
        n_dev = torch.cuda.device_count() if self.backend == "gloo" else 0
        self.device = self.local % n_dev if n_dev else self.local
        self.cdev = "cpu" if self.backend == "gloo" else f"cuda:{self.device}"
        # DC_FORCE_DIST=1: the RCCL path at world size 1 (torch.distributed.run
        # --nproc-per-node 1), to exercise it on a single-GPU box
        if self.world > 1 or os.environ.get("DC_FORCE_DIST") == "1":
            import torch.distributed as dist
            torch.cuda.set_device(self.device)
            dist.init_process_group(self.backend)
            self.dist = dist

    def sync(self):
        if self.dist is not None:
            self.dist.barrier()
        if self.torch.cuda.is_available():
            self.torch.cuda.synchronize()

    def allreduce_u64(self, arr):
        if self.dist is None:
            return arr
        t = self.torch.tensor(arr.astype(np.int64), device=self.cdev)
        self.dist.all_reduce(t)  # RCCL over xGMI
        return t.cpu().numpy().astype(np.uint64)

    def max(self, x):
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def perft_step(eng, d, args, pos, depth, rules=dchess.RULES_REF):
    """One perft: this rank's strided shard of the ply-`split` frontier on its
    GPU, then the per-root-move all-reduce (RCCL) -- dchess/dist.py."""
    return sharded_perft(lambda p, depth, split, r, w: eng.perft_shard(p, depth, split, r, w, rules=rules), pos,
                         depth, args.split, d.rank, d.world, reduce=d.allreduce_u64)


def host_cores():
    """CPU cores this process may use on the box: its affinity mask, capped by the
    box's per-GPU CPU share (OMP_NUM_THREADS is set to it there; os.cpu_count()
    shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else n


def cpu_baselines(args, threads, replay_host=None):
    """Reference-faithful CPU path (refcpu, the restatement of chess.rs) and the
    fast mailbox engine (fastcpu), each on 1 core and on `threads` cores, on
    bounded samples (~30 s of host work in total).  Test infrastructure only:
    never the thing measured as `value`.  The refcpu replay sample is also a
    parity check: its bitmap and digests must equal the GPU's first games."""
    import oracle_lib as O
    out = {}
    root = O.startpos_cells()

    def ref_perft_slice(k, th):
        # refcpu brute-force perft (4096 validate_move calls per interior node) over
        # the perft(4) subtrees of the first k root moves of startpos (a slice of perft(5))
        t0 = time.perf_counter()
        leaves = done = 0
        for m in range(4096):
            fx, fy, tx, ty = (m >> 6) >> 3, (m >> 6) & 7, (m & 63) >> 3, m & 7
            v, cells, turn, _ = O.ref_apply(root, 0, "", fx, fy, tx, ty)
            if v != 0:
                continue
            leaves += O.ref_perft(cells, turn, 4, threads=th)[0]
            done += 1
            if done == k:
                break
        dt = time.perf_counter() - t0
        return {"value": leaves / dt, "unit": "leaf nodes/s", "cores": th, "kind": "port",
                "sample": "refcpu (literal C++ restatement of chess.rs with its per-call board clones, brute force "
                          f"over all 4096 (from,to) pairs per node): perft(4) below the first {k} root moves of "
                          f"startpos (a slice of perft(5)) = {leaves} leaves in {dt:.2f}s",
                "host_cpus_visible": os.cpu_count()}

    out["cpu_baseline"] = ref_perft_slice(6, threads)
    out["cpu_baseline_1core"] = ref_perft_slice(1, 1)
    for th, depth, key in ((threads, args.depth, "cpu_fast"), (1, min(args.depth, 6), "cpu_fast_1core")):
        t0 = time.perf_counter()
        fl, _, _ = O.fast_perft(O.Pos(), depth, O.REF, threads=th)
        dt = time.perf_counter() - t0
        out[key] = {"value": fl / dt, "unit": "leaf nodes/s", "cores": th, "kind": "port",
                    "sample": f"fastcpu mailbox engine (bulk counting) perft(startpos,{depth}) = {fl} leaves "
                              f"in {dt:.2f}s"}
    if not args.no_replay:
        for th, n, key in ((threads, 400_000, "cpu_replay"), (1, 25_024, "cpu_replay_1core")):
            mv = O.fast_gen_games(0x5EED20241022, 0, n, args.plies, 32, threads=threads)
            t0 = time.perf_counter()
            rbm, rdg, st = O.ref_replay(mv, threads=th)
            dt = time.perf_counter() - t0
            out[key] = {"value": float(st[0]) / dt, "unit": "validated moves/s", "cores": th, "kind": "port",
                        "sample": f"refcpu replay of the first {n} seeded games x {args.plies} plies "
                                  f"({int(st[0])} validated moves) in {dt:.2f}s"}
            if replay_host is not None:
                bmh, dgh = replay_host
                w = n // 64
                same = bool((rbm == bmh[:, :w]).all() and (rdg == dgh[:n]).all())
                out[key]["gpu_parity"] = f"bitmap + digests of the GPU's first {n} games == refcpu: {same}"
                if not same:
                    raise SystemExit(f"parity failure: refcpu replay of the first {n} games differs from the GPU")
    return out


REPEAT_BATCH = 8  # runs per batch graph of dc_perft_repeat_device (dc_api.hip kRepeatBatch)


_ENGINES = {}


def perft_contexts(eng, d, n):
    """`eng` plus n - 1 more contexts (streams) on this rank's GPU, kept for the
    whole bench (their level buffers and captured graphs are reused)."""
    extra = _ENGINES.setdefault(d.device, [])
    while len(extra) < n - 1:
        extra.append(dchess.Engine(d.device))
    return [eng] + extra[:n - 1]


def perft_streams(args, depth, world=1):
    """Contexts a repeated perft(depth) is spread over.  One perft's front end
    (round 6: one k_front launch, ~45 us at perft(7), ~22 us at perft(6)) does
    not fill the GPU; with the steps split over two or three contexts --
    streams -- one run's front end executes while another's final stage holds
    the CUs (tools/overlap_perft.py, profiles/r06/overlap_ctx.jsonl, overlap_q:
    perft(7) 0.376 -> 0.351 ms per step with 2, 0.353 with 3, 0.361-0.365 with 4
    (profiles/r06/perft7_streams.txt); perft(6) 0.048 ->
    0.036 with 2 or 3).  A rank of N >= 4 holds a shard whose final stage is
    about as long as its front end, so perft(7) takes 3 there (shard 0 of 8:
    0.085 ms on one context, 0.064 on two).  Every step is still a whole perft
    (of this rank's shard) with its own result record; the bench line also
    reports the one-context figures (perft_one_stream).  Deep runs (the final
    stage is everything) keep one."""
    if args.perft_streams:
        return args.perft_streams
    return 3 if depth <= 6 else (3 if world >= 4 else 2) if depth == 7 else 1


def enqueue_split(engs, steps, base_ptr, W, fn):
    """fn(engine, n_runs, device_address) for each context's share of `steps`
    runs, its records at consecutive slots of the one result array."""
    n = len(engs)
    k0 = 0
    for i, e in enumerate(engs):
        k = steps // n + (1 if i < steps % n else 0)
        if k:
            fn(e, k, base_ptr + k0 * W * 8)
        k0 += k
    for e in engs:
        e.synchronize()


def timed_perft(eng, d, args, pos, depth, steps, warmup, rules=dchess.RULES_REF, want=None, streams=None):
    """warmup + exactly `steps` timed perft(depth) steps (barrier + device sync on
    both sides, max over ranks), parity-checked against the golden count.

    Every timed step is a full perft of this rank's shard, enqueued with
    dc_perft_repeat_device (the captured launch graph, no host round trip
    between steps; each step's result stays on the device).  With N > 1 ranks
    the exchange step -- the all-reduce of each step's per-root-move vector --
    runs over RCCL on the device, bucketed into one collective after the last
    step (K x 258 x 8 B instead of K tiny ones); the reduced totals are checked
    after the timed region."""
    if want is None and rules == dchess.RULES_REF:
        want = REF_STARTPOS.get(depth)
    for _ in range(warmup):  # host path: also captures the launch graph for this shard
        tot, _, _ = perft_step(eng, d, args, pos, depth, rules)
        if want is not None and tot != want:
            raise SystemExit(f"parity failure: perft({depth}) = {tot}, expected {want}")
    W = 258  # divide[256], n_root | overflow << 32, total
    # the first dc_perft_repeat_device call of a configuration runs one plain
    # perft and captures the launch graphs (one run, and a batch of
    # REPEAT_BATCH runs): do it here, outside the timed region
    n_ctx = streams if streams is not None else perft_streams(args, depth, d.world)
    engs = perft_contexts(eng, d, max(1, min(n_ctx, steps)))
    share = -(-steps // len(engs))
    warm = eng.alloc(REPEAT_BATCH * W * 8)
    for e in engs:  # every context captures its graphs (one run; a batch of REPEAT_BATCH when its share has one)
        for nw in ((1, REPEAT_BATCH) if share >= REPEAT_BATCH else (1,)):
            e.perft_repeat_device(pos, depth, args.split, d.rank, d.world, nw, warm, rules=rules)
        e.synchronize()
    warm.free()

    def run(e, k, ptr):
        e.perft_repeat_device(pos, depth, args.split, d.rank, d.world, k, ptr, rules=rules)

    if d.dist is None:
        buf = eng.alloc(steps * W * 8)
        if len(engs) > 1:  # one untimed pass of the split (the first concurrent graph launches run slower)
            enqueue_split(engs, steps, buf.ptr.value, W, run)
        d.sync()
        t0 = time.perf_counter()
        enqueue_split(engs, steps, buf.ptr.value, W, run)
        d.sync()
        dt = time.perf_counter() - t0
        res = buf.download(np.uint64, steps * W).reshape(steps, W)
        buf.free()
        totals = res[:, 257]
    else:
        torch = d.torch
        t = torch.zeros((steps, W), dtype=torch.int64, device=f"cuda:{d.device}")
        if len(engs) > 1:  # one untimed pass of the split, as above
            enqueue_split(engs, steps, t.data_ptr(), W, run)
            t.zero_()
        d.sync()
        t0 = time.perf_counter()
        enqueue_split(engs, steps, t.data_ptr(), W, run)
        # the exchange step of every timed perft, bucketed: one RCCL all-reduce
        # (over xGMI) of all steps' per-root-move vectors, n_root words and totals
        if d.cdev == "cpu":  # gloo rehearsal: the collective on a host copy
            tc = t.cpu()
            d.dist.all_reduce(tc)
            t.copy_(tc)
        else:
            d.dist.all_reduce(t)
        d.sync()
        dt = d.max(time.perf_counter() - t0)
        res = t.cpu().numpy().view(np.uint64)
        totals = res[:, 257]
    if (res[:, 256] >> np.uint64(32)).any():
        raise SystemExit(f"perft({depth}) overflowed its level buffers in the timed region")
    if want is not None and not (totals == want).all():
        raise SystemExit(f"parity failure in timed region: {totals.tolist()} != {want}")
    return int(totals.sum(dtype=np.uint64)), dt


def profiled_perft(eng, d, args, pos, depth, steps):
    """The same steps again with HIP events around every launch on the context's
    stream (dc_ctx_set_profiling) -> per-kernel durations for the roofline."""
    eng.reset_stats()
    eng.set_profiling(True)
    for _ in range(steps):
        perft_step(eng, d, args, pos, depth)
    d.sync()
    eng.set_profiling(False)
    return {k: eng.kernel_stats(k) for k in ("front", "expand_top", "expand_count", "scan", "expand_write", "level_moves",
                                             "count2")}


def _pmc(key):
    """The committed PMC record (profiles/pmc_latest.json) of one kernel, or None."""
    pmc = os.path.join(REPO, "profiles", "pmc_latest.json")
    if not os.path.exists(pmc):
        return None
    return json.load(open(pmc)).get(key)


def valu_roof(kernel, rate, unit_name, w_frozen, pmc_rec, w_key=None):
    """Bound: int32 VALU issue.  With W = VALU lane-ops per unit
    executed by THIS kernel (rocprofv3 SQ_INSTS_VALU x 64 / units, committed
    under profiles/) and the kernel's live rate (HIP events, units/s):
      frac              = rate x W / peak: the fraction of the issue peak the
                          kernel's VALU instructions occupy (full EXEC assumed);
      frac_active_lanes = frac x VALUUtilization (SQ_THREAD_CYCLES_VALU /
                          (SQ_ACTIVE_INST_VALU x 64)): lane-ops actually done;
      frac_int          = rate x W_int / peak with W_int = (SQ_INSTS_VALU_INT32 +
                          SQ_INSTS_VALU_INT64) x 64 / units: SURVEY §8d's and
                          BASELINE.md §3's INT32 VALU fraction;
      valu_slot_occupancy = the VALU issue slots the kernel takes per SIMD
                          ((SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / 1024: one
                          quad-cycle per single instruction or dual-issued pair)
                          x 4.34 cycles each (the measured single-issue cost at
                          4 waves/SIMD, tools/ubench/dual_issue.hip,
                          profiles/r04/issue_costs.json) / the kernel's SIMD
                          cycles at 2.4 GHz: ~1 means the VALU issue slots are
                          all taken (bound by instruction count and pairing);
      dual_issue_frac   = 2 x SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU: the share of
                          VALU instructions issued as a pair (gfx950 pairs only
                          simple ops -- add/sub/and/or/xor/mov/not/bitop3 -- of
                          two waves; shifts, popcounts, selects, 3-source adds
                          are single-issue).
    W_frozen (the first parity-passing kernel's W) is reported
    beside them as the algorithmic gain W_frozen / W, not as a roofline."""
    w = None
    if pmc_rec:
        w = pmc_rec.get("valu_lane_ops_per_unit") or (pmc_rec.get(w_key) if w_key else None)
    measured = w is not None
    w = w if measured else w_frozen
    peak = VALU_PEAK_LANE_OPS
    # without a PMC record of THIS kernel there is no W: frozen W (an upper bound
    # on the work of the first parity kernel) would overstate the fraction
    roof = {"bound": "valu", "kernel": kernel, "unit": "TOPS (int32 VALU lane-ops/s)",
            "achieved": rate * w / 1e12 if measured else None, "peak": peak / 1e12,
            "frac": rate * w / peak if measured else None,
            f"W_lane_ops_per_{unit_name}": w,
            "W_source": pmc_rec["source"] if measured else "frozen (no PMC record for this kernel)",
            f"W_frozen_per_{unit_name}": w_frozen,
            "algorithmic_gain_vs_frozen_W": w_frozen / w if (measured and w_frozen) else None,
            "traffic": pmc_rec.get("hbm_bytes_per_launch") if pmc_rec else None}
    if pmc_rec:
        util = pmc_rec.get("valu_utilization")
        w_int = pmc_rec.get("int_lane_ops_per_unit")
        if util is not None and measured:
            roof["valu_utilization"] = util
            roof["frac_active_lanes"] = roof["frac"] * util
        if w_int is not None:
            roof[f"W_int_lane_ops_per_{unit_name}"] = w_int
            roof["frac_int"] = rate * w_int / peak
        for k in ("lds_conflict_per_lds_cycle", "wait_frac", "salu_per_valu", "dual_issue_frac"):
            if k in pmc_rec:
                roof[k] = pmc_rec[k]
        slots = pmc_rec.get("valu_issue_slots_per_launch")
        units = pmc_rec.get("units_per_dispatch")
        if slots and units and rate:
            # SIMD cycles of one launch at the live rate: units / rate seconds x 2.4 GHz
            roof["valu_slot_occupancy"] = slots * ISSUE_SLOT_CYCLES / (units / rate * CLOCK_HZ)
    return roof


def replay_roof(kr, n_games):
    """k_replay_ref4 (A/B build: DC_REPLAY=1 k_replay_ref, =3 k_replay_ref3).  HBM: 2 B in
    (u16 move) + 1/8 B out (accept bit) per validated move, plus 8 B of digest per game."""
    ab = os.environ.get("DC_REPLAY") if os.environ.get("DCHESS_LIB") else None
    kernel = {"1": "k_replay_ref", "3": "k_replay_ref3"}.get(ab, "k_replay_ref4")
    rec = _pmc("replay")
    if rec and rec.get("kernel", "").split("<")[0].replace("dc::", "") != kernel:
        rec = None
    roof = valu_roof(kernel, kr, "move", W_REPLAY, rec, "valu_lane_ops_per_move")
    roof["hbm"] = {"algorithmic_bytes_per_move": 2.125, "achieved_GBps": kr * 2.125 / 1e9,
                   "peak_GBps": HBM_PEAK_GBPS, "frac": kr * 2.125 / 1e9 / HBM_PEAK_GBPS}
    return roof


def roofline(ks, depth, world):
    """Dominant kernel = the REF final stage (k_count3c: the last three plies, ~90 % of a step).
    traffic = HBM bytes per launch from the PMC passes (2 x FETCH_SIZE + WRITE_SIZE).
    The HBM side: algorithmic bytes = frontier positions x 40 B read per launch."""
    c2 = ks["count2"]
    avg_s = c2["total_ms"] / max(c2["launches"], 1) / 1e3
    leaves = c2["units"] / max(c2["launches"], 1)
    rate = leaves / avg_s if avg_s > 0 else 0.0
    rec = _pmc(f"final_d{depth}") if world == 1 else None
    if rec and FINAL_KERNEL not in rec.get("kernel", ""):
        rec = None  # PMC of another final-stage kernel
    roof = valu_roof(FINAL_KERNEL, rate, "leaf", W_COUNT2, rec, "valu_lane_ops_per_leaf")
    roof.update({"kernel_avg_ms": avg_s * 1e3, "kernel_leaves_per_s": rate})
    if FINAL_KERNEL == "k_count3c":
        # one u32 move word per final-stage parent (ply depth-2) plus its grandparent's board and root
        # tag (34 B per ply depth-3 node); the parents themselves never touch HBM as boards
        alg_bytes = REF_STARTPOS[depth - 2] / world * 4 + REF_STARTPOS[depth - 3] / world * 34
    else:
        frontier = REF_STARTPOS[depth - 2] / world  # ply depth-2 positions read by one launch (exact at N=1)
        alg_bytes = frontier * POS_BYTES
    roof["hbm"] = {"algorithmic_bytes_per_launch": alg_bytes, "achieved_GBps": alg_bytes / avg_s / 1e9,
                   "peak_GBps": HBM_PEAK_GBPS, "frac": alg_bytes / avg_s / 1e9 / HBM_PEAK_GBPS}
    return roof


def _golden_replay():
    path = os.path.join(REPO, "tests", "golden", "replay_golden.json")
    return json.load(open(path)) if os.path.exists(path) else {}


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def replay_leg(eng, d, args):
    """BASELINE configs[3] (C4) at N = 1: 10M seeded games x 80 ply slots; at
    N > 1 configs[4] (C5): 100M games in total, each rank replaying its
    dc_replay_shard_range range (whole 64-game words).  Inputs are generated on
    the device and resident before the timed region.  After it: the exchange
    step (counters all-gathered and folded, bitmaps gathered to rank 0,
    dchess/dist.py) and the parity check of the whole batch's bitmap SHA-256,
    digests and counters against tests/golden/replay_golden.json (fastcpu over
    every game, refcpu on 100k-game samples)."""
    import dchess.dist as D
    torch = d.torch
    n_total = args.games if d.world == 1 else args.c5_games
    first, n = D.replay_range(n_total, d.rank, d.world)
    plies = args.plies
    w_r = (n + 63) // 64
    d_moves = eng.alloc(max(n * plies * 2, 2))
    d_dg = eng.alloc(max(n * 8, 8))
    # the bitmap is a torch tensor so the gather can read it in place (RCCL)
    bm = torch.zeros((plies, max(w_r, 1)), dtype=torch.int64, device=f"cuda:{d.device}") if d.dist is not None \
        else eng.alloc(max(plies * w_r * 8, 8))
    bm_ptr = bm.data_ptr() if d.dist is not None else bm
    seed = 0x5EED20241022
    # end to end (generation included): untimed warmup, then timed
    eng.gen_games_device(d_moves, seed, first, n, plies, 32)
    st = eng.replay_device(d_moves, n, plies, bm_ptr, d_dg)
    d.sync()
    t0 = time.perf_counter()
    for _ in range(args.replay_steps):
        eng.gen_games_device(d_moves, seed, first, n, plies, 32)
        eng.replay_device(d_moves, n, plies, bm_ptr, d_dg)
    d.sync()
    e2e_dt = d.max(time.perf_counter() - t0)
    # replay alone, inputs resident in HBM: the reported rate
    d.sync()
    t0 = time.perf_counter()
    validated = 0
    for _ in range(args.replay_steps):
        st = eng.replay_device(d_moves, n, plies, bm_ptr, d_dg)
        validated += st["validated"]
    d.sync()
    rdt = d.max(time.perf_counter() - t0)
    eng.reset_stats()
    eng.set_profiling(True)
    for _ in range(args.replay_steps):
        eng.replay_device(d_moves, n, plies, bm_ptr, d_dg)
        eng.gen_games_device(d_moves, seed, first, n, plies, 32)
    eng.set_profiling(False)
    rk, gk = eng.kernel_stats("replay"), eng.kernel_stats("gen_games")
    # ---- exchange step + parity (after the timed region)
    stats, whole = D.combine_replay(st, bm if d.dist is not None else None, n_total, d.rank, d.world,
                                    device=d.cdev)
    tot_validated = stats["validated"] * args.replay_steps
    out = {"value": tot_validated / rdt, "unit": "validated moves/s",
           "workload": f"{n_total} seeded games x {plies} ply slots in total (seed 0x5EED20241022, 1/8 junk moves), "
                       + ("one GPU (BASELINE configs[3])" if d.world == 1 else
                          f"game ids split into {d.world} contiguous whole-word ranges (BASELINE configs[4])"),
           "scaling": "weak" if d.world == 1 else "strong", "ms_per_step": 1e3 * rdt / args.replay_steps,
           "validated_per_step": stats["validated"], "combined_stats": stats}
    avg_s = rk["total_ms"] / max(rk["launches"], 1) / 1e3
    kr = (rk["units"] / max(rk["launches"], 1)) / avg_s if avg_s > 0 else 0.0
    out.update({"kernel_avg_ms": avg_s * 1e3, "kernel_moves_per_s": kr, "roofline": replay_roof(kr, n)})
    gen_ms = gk["total_ms"] / max(gk["launches"], 1)
    out["end_to_end"] = {"value": tot_validated / e2e_dt, "unit": "validated moves/s",
                         "ms_per_step": 1e3 * e2e_dt / args.replay_steps, "gen_kernel_avg_ms": gen_ms,
                         "note": "each step generates the games on the device (k_gen_games_ref) and replays them"}
    grec = _pmc("gen_games") if d.world == 1 else None
    if grec and gen_ms > 0:
        out["end_to_end"]["gen_roofline"] = valu_roof("k_gen_games_ref", st["validated"] / (gen_ms / 1e3), "move",
                                                      None, grec)
    g = _golden_replay()
    want = (g.get("c4") if n_total == 10_000_000 else g.get("c5") if n_total == g.get("c5", {}).get("n_games") else None)
    parity = "no golden for this size"
    host = None
    if d.rank == 0 and want is not None:
        if stats != want["stats"]:
            raise SystemExit(f"replay parity failure: counters {stats} != golden {want['stats']}")
        if d.world == 1:
            bmh = bm.download(np.uint64, plies * w_r).reshape(plies, w_r)
            dgh = d_dg.download(np.uint64, n)
            if _sha(dgh) != want["digests_sha256"]:
                raise SystemExit("replay parity failure: per-game digests differ from the golden")
            host = (bmh, dgh)
        else:
            bmh = whole
        if want.get("bitmap_sha256") and _sha(bmh) != want["bitmap_sha256"]:
            raise SystemExit("replay parity failure: accept bitmap differs from the golden")
        parity = "golden"
    out["replay_parity"] = parity
    for b in (d_moves, d_dg):
        b.free()
    if d.dist is None:
        bm.free()
    return out, host


def _latency(eng, calls):
    pos = np.array([dchess.startpos()], dchess.POS_DTYPE)
    mv = np.array([dchess.move_pack(1, 4, 3, 4)], np.uint16)  # e2e4
    for _ in range(50):
        eng.validate_batch(pos, mv)
    ts = np.empty(calls)
    for i in range(calls):
        t0 = time.perf_counter()
        v = eng.validate_batch(pos, mv)
        ts[i] = time.perf_counter() - t0
    if int(v[0]) != dchess.V_OK:
        raise SystemExit("parity failure: e2e4 from startpos rejected")
    us = ts * 1e6
    return {"calls": calls, "median_us": float(np.median(us)), "p99_us": float(np.percentile(us, 99)),
            "min_us": float(us.min())}


def validate_latency(eng, calls=2000):
    """The live consensus call: one dc_validate_batch with n = 1 (is_valid_tx
    validates one move per block, core/src/consensus/hotstuff.rs:138; types.rs:10),
    host buffers in and out.  Per-call wall time over `calls` calls, two ways:
      launched: the batch staged in a pinned block the kernel reads and writes
                in place, one launch, completion seen through a flag the kernel
                publishes there (no stream sync) -- the default path;
      live:     dc_live_validator on a second context: one resident wave polls
                a pinned mailbox (no launch per call)."""
    out = _latency(eng, calls)
    out.update({"unit": "microseconds per dc_validate_batch(n=1) call",
                "note": "launched path (default): pinned in-place I/O, one launch, a completion flag; the "
                        "reference's liveness budget is the 10 s view timeout (core/src/main.rs:30)"})
    live = dchess.Engine(eng.device)
    try:
        live.live_validator(1_000_000)
        out["live"] = _latency(live, calls)
        out["live"]["note"] = ("dc_live_validator (1 s lease): one resident wave serves the call from a pinned, "
                               "stamped mailbox -- a host store and a poll, no launch")
    finally:
        live.live_validator(0)
        live.close()
    # the same two paths from a compiled caller (tools/latency_probe.cpp, built
    # by __graft_entry__.build): how the Rust replica calls the C ABI; Python's
    # ctypes adds ~3 us per call to the figures above
    probe = os.path.join(REPO, "tools", "latency_probe")
    if os.path.exists(probe):
        try:
            p = subprocess.run([probe, "5000"], capture_output=True, text=True, timeout=120)
            r = json.loads(p.stdout.strip().splitlines()[-1])
            if r.get("parity") is not True:
                raise SystemExit("parity failure: latency_probe verdicts")
            out["c_abi"] = {"launched": r["launched"], "live": r["live"], "calls": r["calls"],
                            "note": "tools/latency_probe: steady_clock around each dc_validate_batch(n=1) call "
                                    "of a compiled C++ caller (no Python between the clock and the ABI)"}
        except (subprocess.SubprocessError, ValueError, KeyError, IndexError) as e:
            out["c_abi"] = {"error": str(e)[:200]}
    return out


def state_hash_leg(eng, d, args):
    """keccak256(serde_json(final GameState)) of every game of a seeded replay
    batch (dc_state_hash_device): the hash a replica compares before voting
    (core/src/consensus/hotstuff.rs:153-166), for a whole batch at once."""
    n, plies = args.hash_games, args.plies
    d_moves = eng.alloc(n * plies * 2)
    d_h = eng.alloc(n * 32)
    eng.gen_games_device(d_moves, 0x5EED20241022, d.rank * n, n, plies, 32)
    blob, off = dchess.pack_names([(f"white{d.rank * n + g}", f"black{d.rank * n + g}") for g in range(n)])
    d_names, d_off = eng.names_device(blob, off)  # raw UTF-8 names resident in HBM; escaped on the GPU per call
    eng.state_hash_device(d_moves, n, plies, d_names, d_off, d_h)
    d.sync()
    t0 = time.perf_counter()
    for _ in range(args.hash_steps):
        eng.state_hash_device(d_moves, n, plies, d_names, d_off, d_h)
    d.sync()
    dt = d.max(time.perf_counter() - t0)
    eng.reset_stats()
    eng.set_profiling(True)
    eng.state_hash_device(d_moves, n, plies, d_names, d_off, d_h)
    eng.set_profiling(False)
    k = eng.kernel_stats("state_hash")
    kms = k["total_ms"] / max(k["launches"], 1)
    kp = eng.kernel_stats("state_hash_replay")  # the replay kernel's per-ply info pass before it (round 5)
    pre_ms = kp["total_ms"] / max(kp["launches"], 1) if kp.get("launches") else 0.0
    rec = _pmc("state_hash") if d.world == 1 else None
    roof = valu_roof("k_state_hash_ref", n / (kms / 1e3), "game", None, rec) if rec else None
    if roof is not None:
        # HBM side: 160 B of moves (80 plies x u16) + ~12 B of names in, 32 B of hash out per game
        roof["hbm"] = {"algorithmic_bytes_per_game": 2 * plies + 32 + 12,
                       "achieved_GBps": n / (kms / 1e3) * (2 * plies + 44) / 1e9, "peak_GBps": HBM_PEAK_GBPS}
    h0 = d_h.download(np.uint8, 32)
    for b in (d_moves, d_h, d_names, d_off):
        b.free()
    total = n * d.world * args.hash_steps
    return {"value": total / dt, "unit": "game state hashes/s", "scaling": "weak",
            "workload": f"{n} seeded games x {plies} ply slots per rank: replay + serde_json(GameState) + keccak256 "
                        "per game (names white<g>/black<g>, start history \"\")",
            "ms_per_step": 1e3 * dt / args.hash_steps, "kernel_avg_ms": kms, "replay_prepass_ms": pre_ms,
            "roofline": roof,
            "note": "inputs resident in HBM (moves, raw UTF-8 names); per call: device-side serde_json escaping of the "
                    "names (k_escape_len, scan, k_escape_write, one 8-byte readback), the replay kernel's per-ply info "
                    "pass (replay_prepass_ms) + the hash kernel (kernel_avg_ms)",
            "first_hash": "0x" + bytes(h0).hex()}


def txsig_leg(eng, d, args):
    """App::validate_signature (core/src/consensus/hotstuff.rs:168-208) + the owner
    check (:141-148) for a resident batch: the 512 signed transactions of
    tests/golden/txsig_batch.json tiled to --txs, parity-checked against the
    fixture's verdicts (dc_verify_tx_batch_device, k_verify_tx)."""
    fx = json.load(open(os.path.join(REPO, "tests", "golden", "txsig_batch.json")))["txs"]
    n = args.txs
    reps = (n + len(fx) - 1) // len(fx)
    blob, off, acts, turns = dchess.pack_txs([(t["white"], t["black"], t["sig"], t["pk"]) for t in fx] * reps,
                                             np.array([t["action"] for t in fx] * reps, np.uint32),
                                             np.array([t["turn"] for t in fx] * reps, np.int8))
    off, acts, turns = off[:4 * n + 1], acts[:n], turns[:n]
    blob = blob[:int(off[-1])]
    want = np.array([t["verdict"] for t in fx] * reps, np.uint8)[:n]
    bufs = []
    for arr in (np.frombuffer(blob, np.uint8), off, acts, turns):
        b = eng.alloc(max(arr.nbytes, 1))
        b.upload(arr)
        bufs.append(b)
    d_v = eng.alloc(n)
    eng.verify_txs_device(*bufs, n, d_v)  # warmup (builds the G table once per context)
    got = d_v.download(np.uint8, n)
    if not (got == want).all():
        raise SystemExit(f"parity failure: {int((got != want).sum())} signature verdicts differ from the fixture")
    d.sync()
    t0 = time.perf_counter()
    for _ in range(args.tx_steps):
        eng.verify_txs_device(*bufs, n, d_v)
    d.sync()
    dt = d.max(time.perf_counter() - t0)
    eng.reset_stats()
    eng.set_profiling(True)
    eng.verify_txs_device(*bufs, n, d_v)
    eng.set_profiling(False)
    k = eng.kernel_stats("verify_tx")
    for b in bufs + [d_v]:
        b.free()
    kms = k["total_ms"] / max(k["launches"], 1)
    out = {"value": n * d.world * args.tx_steps / dt, "unit": "transaction signature checks/s", "scaling": "weak",
           "workload": f"{n} transactions per rank (512 distinct client-signed txs tiled; compressed secp256k1 keys; "
                       "26 % rejected): serde_json message + SHA-256 + hex/key parse + ECDSA verify + owner check",
           "ms_per_step": 1e3 * dt / args.tx_steps, "kernel_avg_ms": kms, "kernel_per_s": n / (kms / 1e3)}
    rec = _pmc("verify_tx")
    if rec and d.world == 1:
        out["roofline"] = valu_roof("k_verify_tx", n / (kms / 1e3), "tx", None, rec)
    return out


def cpu_txsig(threads):
    """The same per-transaction code compiled for the host (build/test_secp, the
    kernel's dc_txsig.h on one core) over a bounded sample of the fixture."""
    import subprocess
    exe = os.path.join(REPO, "distributed-chess_amd", "build", "test_secp")
    if not os.path.exists(exe):
        return None
    fx = json.load(open(os.path.join(REPO, "tests", "golden", "txsig_batch.json")))["txs"][:256]
    h = lambda s: s.encode().hex() or "-"  # noqa: E731
    lines = "".join(f"tx {h(t['white'])} {h(t['black'])} {' '.join(map(str, t['action']))} {h(t['sig'])} "
                    f"{h(t['pk'])} {t['turn']}\n" for t in fx)
    reps = 8
    # the binary times its own verify loop (steady_clock around the checks only:
    # no process start-up, parsing or G-table build inside the clock)
    p = subprocess.run([exe], input=f"timed {reps}\n" + lines + "end\n", capture_output=True, text=True, timeout=300)
    out = p.stdout.split()
    ns = int(out[out.index("ns") + 1])
    got = [int(x) for x in out[:out.index("ns")]]
    if got != [t["verdict"] for t in fx]:
        raise SystemExit("parity failure: host build of k_verify_tx's code disagrees with the fixture")
    if ns <= 0:
        raise SystemExit("cpu_txsig: non-positive elapsed time from build/test_secp")
    return {"value": reps * len(fx) / (ns * 1e-9), "unit": "transaction signature checks/s", "cores": 1,
            "kind": "port",
            "sample": f"host build of dc_txsig.h (clang -O2, 32-bit limbs), {reps} passes over {len(fx)} fixture "
                      "transactions on one core, timed inside the binary around the verify loop only; the "
                      "reference's libsecp256k1 could not be built here"}


LEGS = ("perft", "perft6", "perft8", "perft9", "fide7", "fidesuite", "replay", "hash", "tx", "latency")
# Published FIDE perft counts (chessprogramming wiki; tests/golden/oracle_golden.json perft_fide),
# the C2/C3/C5 configurations under standard rules, which the reference cannot compute.
_OG = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_golden.json")))["perft_fide"]
FIDE_SUITE = ("startpos", "kiwipete", "pos3", "pos4", "pos5", "pos6")


def concurrent_perfts(d, args, items, depth, steps, rules):
    """The positions of a suite timed as one batch: one context -- one stream
    -- per position, every position's `steps` repeat runs enqueued before any
    is waited for, so the small per-position launch sequences (a depth-5 FIDE
    final stage has 3k-100k parents) fill the GPU together instead of one
    after another.  Returns (leaves, wall seconds); every step of every
    position is checked against its published count after the timed region."""
    W = 258
    engs, bufs = [], []
    for pos, want in items:
        e = dchess.Engine(d.device)
        engs.append(e)
        tot, _, _ = e.perft(pos, depth, rules=rules)  # warm-up, parity
        if tot != want:
            raise SystemExit(f"parity failure: FIDE perft({depth}) = {tot}, expected {want}")
        b = e.alloc(max(REPEAT_BATCH, steps) * W * 8)
        for nw in (1, REPEAT_BATCH):  # graph captures (the one-run and the batch graph)
            e.perft_repeat_device(pos, depth, args.split, 0, 1, nw, b, rules=rules)
        e.synchronize()
        bufs.append(b)
    for (pos, _), e, b in zip(items, engs, bufs):  # one untimed concurrent pass
        e.perft_repeat_device(pos, depth, args.split, 0, 1, steps, b, rules=rules)
    for e in engs:
        e.synchronize()
    d.sync()
    t0 = time.perf_counter()
    for (pos, _), e, b in zip(items, engs, bufs):
        e.perft_repeat_device(pos, depth, args.split, 0, 1, steps, b, rules=rules)
    for e in engs:
        e.synchronize()
    d.sync()
    dt = time.perf_counter() - t0
    leaves = 0
    for (pos, want), e, b in zip(items, engs, bufs):
        res = b.download(np.uint64, steps * W).reshape(steps, W)
        if not (res[:, 257] == want).all():
            raise SystemExit(f"parity failure in a concurrent FIDE step: {res[:, 257][:4]} != {want}")
        leaves += want * steps
        b.free()
        e.close()
    return leaves, dt


SUITE_STREAMS = 2


def batch_perfts(eng, d, args, items, depth, steps, rules):
    """The positions of a suite as ONE tree (dc_perft_batch_repeat_device: same side
    to move, root moves sharing the divide tags), so every level and the final
    stage run one grid over all positions.  Returns (leaves, wall seconds,
    final-stage kernel ms of one profiled batch run); every step's per-position
    totals (divide summed over dc_perft_batch's root_pos) are checked against the
    published counts after the timed region."""
    W = 258
    pos = [p for p, _ in items]
    want = [w for _, w in items]
    tot, div, rm, rp = eng.perft_batch(pos, depth, rules=rules)  # warm-up, parity, the root-move owners
    if [int(x) for x in tot] != want:
        raise SystemExit(f"parity failure: batch FIDE perft({depth}) = {list(tot)}, expected {want}")
    b = eng.alloc(max(REPEAT_BATCH, steps) * W * 8)
    # the steps over SUITE_STREAMS contexts.  (Round 6: four measured 0.297-0.312
    # ms per step against 0.330 on two in a process that ran only this leg, but
    # 0.332 against 0.331 after the perft legs had run on the same contexts,
    # as the default bench does, and 0.326-0.329 on four fresh contexts:
    # profiles/r06/suite_streams.txt; so two.)
    engs = perft_contexts(eng, d, max(1, min(args.perft_streams or SUITE_STREAMS, steps)))

    def run(e, k, ptr):
        e.perft_batch_repeat_device(pos, depth, args.split, k, ptr, rules=rules)

    for e in engs:
        for nw in (1, REPEAT_BATCH):  # graph captures (the one-run and the batch graph)
            run(e, nw, b.ptr.value)
    enqueue_split(engs, steps, b.ptr.value, W, run)  # one untimed pass
    d.sync()
    t0 = time.perf_counter()
    enqueue_split(engs, steps, b.ptr.value, W, run)
    d.sync()
    dt = time.perf_counter() - t0
    res = b.download(np.uint64, steps * W).reshape(steps, W)
    b.free()
    nr = len(rp)
    for r in range(steps):
        per = [int(res[r, :nr][rp == i].sum()) for i in range(len(pos))]
        if per != want:
            raise SystemExit(f"parity failure in a batch FIDE step: {per} != {want}")
    eng.reset_stats()
    eng.set_profiling(True)
    eng.perft_batch(pos, depth, rules=rules)
    d.sync()
    eng.set_profiling(False)
    ks = eng.kernel_stats("count2")
    return sum(want) * steps, dt, ks["total_ms"], ks["launches"]


def fide_leg(eng, d, args, name, depth, keys, pmc_key):
    """FIDE perft (DC_RULES_FIDE: castling, en passant, promotion, no self-check)
    of one or more positions, each timed like the headline (dc_perft_repeat_device
    steps, parity against the published table) and summed: value = all leaves /
    all timed wall time.  The final stage is k_count2b (FIDE: the last ply bulk
    counted per child with pin/check masks; DESIGN.md section 3.2 says why the
    REF two-ply split cannot apply)."""
    steps = max(2, args.steps // 4)
    leaves, dt, per = 0, 0.0, {}
    kms, kunits, kl = 0.0, 0, 0
    batched = len(keys) > 1 and d.dist is None
    for k in ([] if batched and args.suite_batch_only else keys):
        pos = dchess.pos_from_fen(_OG[k]["fen"])
        want = _OG[k]["perft"][str(depth)]
        lv, t = timed_perft(eng, d, args, pos, depth, steps, 1, rules=dchess.RULES_FIDE, want=want)
        leaves += lv
        dt += t
        per[k] = {"leaves": want, "ms_per_step": 1e3 * t / steps}
        # the final stage's kernel time of one step (profiled run, outside the timed region)
        eng.reset_stats()
        eng.set_profiling(True)
        perft_step(eng, d, args, pos, depth, dchess.RULES_FIDE)
        d.sync()
        eng.set_profiling(False)
        ks = eng.kernel_stats("count2")
        kms += ks["total_ms"]
        kl += ks["launches"]
        kunits += want // d.world
    seq_ms = 1e3 * dt / steps
    if batched and args.suite_batch_only:
        kunits = sum(_OG[k]["perft"][str(depth)] for k in keys) // d.world
    how = None
    if batched:  # the suite as one batch: the leg's value
        items = [(dchess.pos_from_fen(_OG[k]["fen"]), _OG[k]["perft"][str(depth)]) for k in keys]
        # whole 8-run batch graphs, at least two
        steps = REPEAT_BATCH * max(2, -(-args.steps // REPEAT_BATCH))
        try:  # one tree (dc_perft_batch): one launch sequence for all positions
            leaves, dt, bkms, bkl = batch_perfts(eng, d, args, items, depth, steps, dchess.RULES_FIDE)
            how = "tree"
            kms, kl = bkms, bkl  # the roofline's kernel: the batch's one final stage
        except dchess.DChessError:  # (more than 256 root moves, or mixed sides to move)
            # one context (stream) per position, longest first (the sequential times
            # above): with more streams than hardware queues (GPU_MAX_HW_QUEUES), a
            # queue shared by two streams pairs a long position with a short one
            order = sorted(keys, key=lambda k: -per[k]["ms_per_step"])
            items = [(dchess.pos_from_fen(_OG[k]["fen"]), _OG[k]["perft"][str(depth)]) for k in order]
            leaves, dt = concurrent_perfts(d, args, items, depth, steps, dchess.RULES_FIDE)
            how = "streams"
    out = {"value": leaves / dt, "unit": "leaf nodes/s", "ms_per_step": 1e3 * dt / steps, "steps": steps,
           "workload": name, "rules": "FIDE", "scaling": "strong", "leaves_per_step": leaves // steps,
           "parity": "published tables (chessprogramming wiki), every timed step", "positions": per,
           "final_kernel_ms": kms}
    if batched:
        out["batch"] = ({"tree": "the positions as one tree (dc_perft_batch_repeat_device: root moves of all "
                                 "positions share the divide tags, every level and the final stage one grid); "
                                 f"final_kernel_ms is that one final stage; the timed steps are split over "
                                 f"{args.perft_streams or SUITE_STREAMS} contexts (streams), each step a whole "
                                 f"batch with its own result record",
                         "streams": "one context (stream) per position, every position's repeat runs enqueued "
                                    "before any wait"}[how] +
                        "; positions[].ms_per_step and sequential_ms_per_step time the positions one after another")
        out["sequential_ms_per_step"] = seq_ms
        if how == "tree":
            out["streams_per_gpu"] = args.perft_streams or SUITE_STREAMS
    rec = _pmc(pmc_key) if d.world == 1 else None
    if rec and kl and kms > 0:
        out["roofline"] = valu_roof("k_count2b", kunits / (kms / 1e3), "leaf", W_COUNT2, rec,
                                    "valu_lane_ops_per_leaf")
        out["roofline"]["kernel_leaves_per_s"] = kunits / (kms / 1e3)
    return out


def perft8_leg(eng, d, args, pos):
    """REF perft(startpos, 8): BFS to ply 5, ply 6 as 64-bit move words and the
    fused three-ply final stage (k_level_moves + k_count3c, as the headline one
    level deeper), timed like the headline and checked
    against the committed golden (tests/golden/ref_deep.json, fastcpu)."""
    deep = os.path.join(REPO, "tests", "golden", "ref_deep.json")
    want = json.load(open(deep)).get("startpos_d8", {}).get("total") if os.path.exists(deep) else None
    if want is not None:
        REF_STARTPOS[8] = want
    steps = max(2, args.steps // 4)
    leaves, dt = timed_perft(eng, d, args, pos, 8, steps, 1)
    eng.reset_stats()
    eng.set_profiling(True)
    perft_step(eng, d, args, pos, 8)
    d.sync()
    eng.set_profiling(False)
    ks = {k: eng.kernel_stats(k) for k in ("count2", "dfs")}
    out = {"value": leaves / dt, "unit": "leaf nodes/s", "ms_per_step": 1e3 * dt / steps, "steps": steps,
           "workload": "perft(startpos, 8) RULES_REF: BFS to ply 5, ply 6 as 64-bit move words, three-ply fused "
                       "final stage (k_count3c)", "scaling": "strong", "leaves_per_step": leaves // steps,
           "parity": "golden (fastcpu, tests/golden/ref_deep.json)" if want is not None else "no golden",
           "path": "k4" if ks["dfs"]["launches"] else "fused"}
    if ks["count2"]["launches"]:
        out["roofline"] = roofline(ks, 8, d.world)
    return out


def perft9_leg(eng, d, args, pos):
    """REF perft(startpos, 9), both ways, each checked against the committed
    golden every step (2,597,923,551,373):
      * default: ply 6 as boards and the fused three-ply final stage over
        slices of 2^21 ply-6 nodes (k_level_moves + k_count3c with 64-bit
        words); its roofline takes W from the perft(8)
        PMC record (the same kernel body, 64-bit words);
      * "k4": K4 (k_perft_dfs: BFS to ply 5, then a per-lane DFS with an
        explicit stack over 2 plies and the two-ply bulk final stage), forced
        with DCHESS_PERFT_K4=1 -- the north star's per-lane-stack path."""
    deep = os.path.join(REPO, "tests", "golden", "ref_deep.json")
    want = json.load(open(deep)).get("startpos_d9", {}).get("total") if os.path.exists(deep) else None
    if want is not None:
        REF_STARTPOS[9] = want

    def run(steps):
        leaves, dt = timed_perft(eng, d, args, pos, 9, steps, 1)
        eng.reset_stats()
        eng.set_profiling(True)
        perft_step(eng, d, args, pos, 9)
        d.sync()
        eng.set_profiling(False)
        return leaves, dt, {k: eng.kernel_stats(k) for k in ("count2", "dfs")}

    steps = 2
    leaves, dt, ks = run(steps)
    parity = "golden (fastcpu, tests/golden/ref_deep.json)" if want is not None else "no golden"
    out = {"value": leaves / dt, "unit": "leaf nodes/s", "ms_per_step": 1e3 * dt / steps, "steps": steps,
           "workload": "perft(startpos, 9) RULES_REF: BFS to ply 6, fused three-ply final stage over slices of "
                       "ply 6 (64-bit move words)", "scaling": "strong", "leaves_per_step": leaves // steps,
           "parity": parity, "path": "k4" if ks["dfs"]["launches"] else "fused-sliced",
           "final_kernel_ms": ks["count2"]["total_ms"]}
    rec = _pmc("final_d8") if d.world == 1 else None
    if rec and ks["count2"]["launches"] and ks["count2"]["total_ms"] > 0:
        rate = (want or leaves // steps) / d.world / (ks["count2"]["total_ms"] / 1e3)
        out["roofline"] = valu_roof("k_count3c", rate, "leaf", W_COUNT2, rec, "valu_lane_ops_per_leaf")
        out["roofline"]["kernel_leaves_per_s"] = rate
        out["roofline"]["W_note"] = "W of the perft(8) record: the same kernel body with 64-bit words"
    os.environ["DCHESS_PERFT_K4"] = "1"
    try:
        l4, dt4, ks4 = run(1)
    finally:
        del os.environ["DCHESS_PERFT_K4"]
    k = ks4["dfs"]
    k4 = {"value": l4 / dt4, "ms_per_step": 1e3 * dt4, "steps": 1, "parity": parity,
          "workload": "K4: BFS to ply 5, per-lane DFS (2 plies) + two-ply bulk final stage",
          "dfs_kernel_ms": k["total_ms"] / max(k["launches"], 1)}
    rec = _pmc("dfs_d9") if d.world == 1 else None
    if rec and k["launches"]:
        rate = k["units"] / max(k["launches"], 1) / (k4["dfs_kernel_ms"] / 1e3)
        k4["roofline"] = valu_roof("k_perft_dfs", rate, "leaf", W_COUNT2, rec, "valu_lane_ops_per_leaf")
        k4["roofline"]["kernel_leaves_per_s"] = rate
    out["k4"] = k4
    return out


def main():
    args = parse()
    d = Dist(args.gpus)
    eng = dchess.Engine(d.device)
    pos = dchess.startpos()

    if args.no_perft and not args.profile_only:
        raise SystemExit("--no-perft is only meaningful with --profile-only")
    if args.only:
        legs = set(args.only.split(","))
        bad = legs - set(LEGS)
        if bad:
            raise SystemExit(f"--only: unknown legs {sorted(bad)} (known: {', '.join(LEGS)})")
        args.profile_only = True
    else:
        legs = set(LEGS)
        if args.no_perft:
            legs -= {"perft"}
        if args.profile_only:  # rocprof passes: headline (or replay + tx with --no-perft) only
            legs -= {"perft6", "perft8", "perft9", "fide7", "fidesuite", "hash", "latency"}
            if not args.no_perft:
                legs -= {"tx"}
        if args.no_replay or args.games <= 0:
            legs -= {"replay"}
        if args.hash_games <= 0:
            legs -= {"hash"}
        if args.txs <= 0:
            legs -= {"tx"}
        if args.depth == 6:
            legs -= {"perft6"}
    # ------------------------------------------------- perft (headline: depth 7)
    p6 = p8 = p9 = None
    leaves, dt, ks = 0, 0.0, None
    def note(leg):  # one progress line per leg on stderr (long profiler passes stay visibly alive)
        if d.rank == 0:
            print(f"[bench] {leg} {time.strftime('%H:%M:%S')}", file=sys.stderr, flush=True)

    if "perft" in legs:
        note("perft")
        leaves, dt = timed_perft(eng, d, args, pos, args.depth, args.steps, args.warmup)
        ks = profiled_perft(eng, d, args, pos, args.depth, args.steps)
    # perft(6) (BASELINE configs[1]) on the same engine and method, secondary
    if "perft6" in legs:
        note("perft6")
        l6, dt6 = timed_perft(eng, d, args, pos, 6, 4 * args.steps, args.warmup)
        p6 = {"value": l6 / dt6, "unit": "leaf nodes/s", "ms_per_step": 1e3 * dt6 / (4 * args.steps),
              "steps": 4 * args.steps, "workload": "perft(startpos, 6) RULES_REF, frontier split at ply 3",
              "scaling": "strong", "streams_per_gpu": perft_streams(args, 6, d.world)}
    # one context (stream) per GPU: one run's latency, its front end not hidden
    # behind another run's final stage (the like-for-like figure)
    one = None
    if "perft" in legs and (not args.profile_only or args.only):
        note("perft_one_stream")
        one = {}
        for dd, k in ((args.depth, args.steps), (6, 4 * args.steps)):
            l1, dt1 = timed_perft(eng, d, args, pos, dd, k, args.warmup, streams=1)
            one[f"perft{dd}"] = {"value": l1 / dt1, "unit": "leaf nodes/s", "ms_per_step": 1e3 * dt1 / k, "steps": k}
    if "perft8" in legs:
        note("perft8")
        p8 = perft8_leg(eng, d, args, pos)
    if "perft9" in legs:
        note("perft9")
        p9 = perft9_leg(eng, d, args, pos)
    f7 = fs = None
    if "fide7" in legs:  # BASELINE configs[4]'s perft(startpos, 7) under standard rules
        note("fide7")
        f7 = fide_leg(eng, d, args, "perft(startpos, 7) RULES_FIDE", 7, ("startpos",), "fide_d7")
    if "fidesuite" in legs:  # BASELINE configs[2]: Kiwipete + the standard suite at depth 5
        note("fidesuite")
        fs = fide_leg(eng, d, args, "Kiwipete + perft suite positions 3-6 + startpos at depth 5, RULES_FIDE", 5,
                      FIDE_SUITE, "fide_suite_d5")

    # --------------------------------------------------------------- replay
    replay = None
    replay_host = None
    if "replay" in legs:
        note("replay")
        replay, replay_host = replay_leg(eng, d, args)

    # ------------------------------------------- state hash
    shash = None
    if "hash" in legs:
        note("hash")
        shash = state_hash_leg(eng, d, args)

    # ------------------------------------ transaction signatures
    txsig = None
    if "tx" in legs:
        note("tx")
        txsig = txsig_leg(eng, d, args)

    v1 = validate_latency(eng) if "latency" in legs else None
    if d.rank != 0 or (args.profile_only and not args.only):
        return
    line = {
        "metric": METRIC, "value": leaves / dt if dt > 0 else 0.0, "unit": "leaf nodes/s",
        "n_gpus": d.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps if dt > 0 else None,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (startpos tree; seeded random-legal games for replay)",
        "config": {"workload": f"perft(startpos, {args.depth}) RULES_REF (bit-exact with core/src/chess.rs), "
                               f"frontier split at ply {args.split} into strided shards over ranks, "
                               "per-root-move counts all-reduced over RCCL",
                   "depth": args.depth, "rules": "REF", "leaves_per_step": REF_STARTPOS.get(args.depth),
                   "parallelism": f"dp{d.world}",
                   "streams_per_gpu": perft_streams(args, args.depth, d.world),
                   "streams_note": "the K timed steps are split over this many contexts (HIP streams) per GPU, "
                                   "each enqueuing its share at once; each step is a whole perft with its own "
                                   "result record, and one run's latency-bound front end overlaps another's "
                                   "final stage"},
    }
    if ks is not None:
        line["roofline"] = roofline(ks, args.depth, d.world)
        line["kernels_ms_per_step"] = {k: v["total_ms"] / args.steps for k, v in ks.items()}
    if one is not None:
        line["perft_one_stream"] = one
    if p8 is not None:
        line["perft8"] = p8
    if p9 is not None:
        line["perft9"] = p9
    if p6 is not None:
        line["perft6"] = p6
    if f7 is not None:
        line["fide_perft7"] = f7
    if fs is not None:
        line["fide_suite_d5"] = fs
    if shash is not None:
        line["state_hash"] = shash
    if replay is not None:
        line["replay"] = replay
    if txsig is not None:
        line["tx_signatures"] = txsig
    if v1 is not None:
        line["validate_n1_latency"] = v1
    if not args.no_cpu and d.world == 1:
        threads = args.cpu_threads or host_cores()
        line.update(cpu_baselines(args, threads, replay_host))
        if txsig is not None:
            ct = cpu_txsig(threads)
            if ct is not None:
                line["tx_signatures"]["cpu_baseline"] = ct
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
