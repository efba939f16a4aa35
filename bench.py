#!/usr/bin/env python3
"""Benchmark of the batched quorum engine (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

One step = one pass of the hot path over this rank's resident batch.  The
headline workload (default, BASELINE configs[1]) is 64M groups x 5-voter
MajorityConfig CommittedIndex + VoteResult (+ TallyVotes counts) per GPU;
groups are sharded across ranks (weak scaling, no data-path collective; one
RCCL all-reduce of the statistics vector after the timed region).

Rank 0 prints ONE JSON line with the metric, the roofline of the dominant
kernel (HIP events on the launch stream), and the CPU baseline (oracle port,
rank 0 at N=1 only, bounded sample).
"""
import argparse
import json
import os
import sys
import time

import subprocess

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

engine = None  # etcd_amd.engine, imported once the process knows its rank

METRIC = "quorum group-evals/sec at 1/2/4/8 MI355X; % HBM peak; speedup vs Go host"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMD32 x 2.4 GHz, one wave64 instruction per
# 2 cycles per SIMD (MI355X_MICROARCH.md: v_fma_f32 wave64 = 2 cyc; the
# 157.3 TFLOPS fp32 vector peak) = 1.2288e12 wave-instructions/s
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2

WORKLOADS = {
    # name: (description, groups per GPU, slots, kind)
    "config2_n5": ("64M groups x 5-voter MajorityConfig CommittedIndex+VoteResult "
                   "(TallyVotes counts into the stats)", 1 << 26, 5, "majority"),
    "config2_n7": ("64M groups x 7-voter MajorityConfig CommittedIndex+VoteResult "
                   "(TallyVotes counts into the stats)", 1 << 26, 7, "majority"),
    "config3_joint": ("128M groups x JointConfig 5+5 (S=10 slots, learners masked, "
                      "shape-bucketed layout) CommittedIndex+VoteResult",
                      1 << 27, 10, "joint"),
    "config3_joint_rot": ("128M groups x JointConfig 5+5 (S=10 slots, learners masked, "
                          "per-group rotated slots) CommittedIndex+VoteResult",
                          1 << 27, 10, "joint_rot"),
    "config3_joint_packed": ("128M groups x JointConfig 5+5 (S=10 slots, learners masked) "
                             "built from per-group ConfStates (overlap uniform 0..5 per group, "
                             "peer IDs in per-group rotated order) through the product packer "
                             "(qe_pack_order shape bucketing + qe_pack_confstate, per 16M-group "
                             "batch) CommittedIndex+VoteResult", 1 << 27, 10, "joint_packed"),
    "config4_repl": ("32M groups x 5 voters lockstep replication round (MaybeUpdate, "
                     "CommittedIndex, term-gated commit, ReadIndex quorum)", 1 << 25, 5, "repl"),
    "config4_repl_joint": ("32M groups x joint 5+5 over 6 slots (replacing one voter: "
                           "C_old {0,1,2,3,4}, C_new {0,1,2,3,5}) lockstep replication round",
                           1 << 25, 6, "repl_joint"),
    "ready_collect": ("64M groups: qe_collect of a Ready-style commit delta (half the groups "
                      "flagged): ascending group ids + their committed index", 1 << 26, 1,
                      "collect"),
    "config5_elec": ("2M groups x 64 fused election steps (5 voters, drop 0.2, grant 0.5)",
                     1 << 21, 5, "elec"),
    "config5_prevote_cq": ("2M groups x 64 fused election steps with PreVote and CheckQuorum "
                           "(5 voters, drop 0.2, grant 0.5, peer active 0.7)", 1 << 21, 5,
                           "elec_pvcq"),
    "progress_step": ("16M groups x 5 peers: one round of MsgAppResp accept/reject + "
                      "MsgHeartbeatResp through the full Progress state machine "
                      "(inflights F=8, leader-log model R=4)", 1 << 24, 5, "progress"),
    "progress_step_n7": ("16M groups x 7 peers: the progress_step round with 6 followers "
                         "(BASELINE config 2's 7-voter shape)", 1 << 24, 7, "progress"),
    "progress_step_joint": ("16M groups x joint 5+5 over 6 slots (one voter replaced: C_old "
                            "{0,1,2,3,4}, C_new {0,1,2,3,5}): the progress_step round, commits "
                            "need both halves", 1 << 24, 6, "progress_joint"),
    "progress_send": ("16M groups x bcastAppend after a proposal (qe_progress_send to the 4 "
                      "followers, StateReplicate, Inflights F=8 with room): one MsgApp and one "
                      "ring entry per peer", 1 << 24, 5, "psend"),
    "heartbeat": ("16M groups x MsgBeat through qe_heartbeat: bcastHeartbeat to the 4 followers "
                  "(Commit = min(Match, committed) per follower, the newest pending ReadIndex "
                  "context of a 0..4-entry queue)", 1 << 24, 5, "heartbeat"),
    "propose": ("16M groups x one MsgProp of 3 entries (24 B of payload) through qe_propose: the "
                "MsgProp gates, increaseUncommittedSize, appendEntry (lastIndex + 3, the leader's "
                "MaybeUpdate, maybeCommit) and bcastAppend to the 4 followers (StateReplicate, "
                "Inflights F=8 with room, noLimit MaxSizePerMsg): one MsgApp and one ring entry "
                "each", 1 << 24, 5, "propose"),
    "switch_config": ("16M groups x switchToConfig after an applied conf change through "
                      "qe_switch_config (leader in slot 0, followers StateReplicate with room, "
                      "old voters {0,1,2,3} + learner 4): half the groups remove voter 3 (the "
                      "smaller quorum commits more: bcastAppend to 1, 2, 4), half promote the "
                      "learner (maybeCommit under 5 voters, else the probe of every peer); a "
                      "transfer to 3 pending in 1/8 of the groups", 1 << 24, 5, "switch"),
    "check_quorum": ("16M groups x 5 peers: MsgCheckQuorum on the leader over the resident "
                     "Progress words (QuorumActive over RecentActive, step-down mask, "
                     "RecentActive reset; each follower active with p = 0.7)", 1 << 24, 5, "cq"),
    "confchange": ("16M groups x Changer.Simple(AddNode(learner), AddLearnerNode(new)) on "
                   "slot masks: promote a learner, add a learner with initProgress "
                   "(3 voters + 1 learner + 1 free slot)", 1 << 24, 5, "confchange"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="config2_n5", choices=sorted(WORKLOADS))
    ap.add_argument("--groups", type=int, default=0, help="override groups per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-aux", action="store_true", help="skip the secondary workloads")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = this process's CPU share: the affinity "
                         "set, capped by OMP_NUM_THREADS when the box sets it)")
    ap.add_argument("--cpu-groups", type=int, default=1 << 21)
    ap.add_argument("--allow-stats-fallback", action="store_true",
                    help="N > 1: accept the stats all-reduce through torch when the engine's "
                         "qe_allreduce_stats path cannot be set up (reported; otherwise exit 3)")
    ap.add_argument("--aux-groups-div", type=int, default=1,
                    help="rehearsal only: divide every secondary workload's group count")
    return ap.parse_args(argv)


def cpu_share():
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def maybe_spawn(args):
    """`bench.py --gpus N` outside a torch.distributed launch starts N ranks
    (one process per GPU) with torch.distributed.run as a CHILD process --
    this process has not touched the GPU -- and exits with its status.
    Rank 0 of the children prints the JSON line."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return False
    # --standalone: the rendezvous store binds a free port itself (a port
    # picked here and released could be taken before the launcher binds it)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone",
           "--local-addr", "127.0.0.1", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


# ABI 8: the Progress workloads keep their Inflights rings in the 16-bit form
# (infl16: 16 bytes per peer, two peers per HBM sector); 0 = the 32-bit
# words of ABI 4 (A/B)
RING16 = os.environ.get("QE_BENCH_RING16", "1") == "1"
COMM_INIT_TIMEOUT_MS = 120_000  # qe_comm_init_timeout: peers that never join
STATS_WAIT_S = 60.0  # bound on one engine all-reduce's completion (its own stream)


class Dist:
    """One process per GPU (torch.distributed.run env).  Collectives go over
    RCCL (backend "nccl") by default: barrier/max through torch, the stats
    all-reduce through the engine's own C ABI (qe_allreduce_stats on an RCCL
    communicator set up with qe_comm_init_timeout -- the path a Go host uses).
    QE_DIST_BACKEND=gloo with QE_DEVICE_MOD=1 rehearses the multi-rank logic
    on a 1-GPU box (all ranks on cuda:0, counters reduced on the host).

    Which path the statistics take is decided ONCE, at start-up, by every
    rank together (_select_stats_path): each rank reports whether its part
    of the engine communicator's set-up succeeded and the ranks take the MIN
    over the torch group, so all of them use qe_allreduce_stats or all of
    them use torch's all_reduce -- never a mix, which would leave the ranks
    in different collectives (a hang).  A fallback is reported in the JSON
    line and fails the run unless --allow-stats-fallback is given.

    Every agreement runs on a host-side gloo group (`hgroup`), never on the
    device: a torch collective on the launch stream could queue behind an
    engine all-reduce that waits for a peer which never enqueued it.  The
    engine all-reduce itself runs on a stream of its own and its completion
    is awaited with a deadline; a failure anywhere aborts the engine
    communicator on every rank before any fallback runs (on the host
    group), so no rank can block behind the aborted collective."""

    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = backend or os.environ.get("QE_DIST_BACKEND", "nccl")
        mod = int(os.environ.get("QE_DEVICE_MOD", "0"))
        dev_idx = self.local % mod if mod > 0 else self.local
        if torch.cuda.is_available():
            torch.cuda.set_device(dev_idx)
            self.dev = torch.device("cuda", dev_idx)
        else:  # CPU tests of the rank logic (gloo)
            self.dev = torch.device("cpu")
        self.comm = None
        self.hgroup = None          # host-side (gloo) group for every agreement
        self.stats_path = None      # what the stats all-reduce went through
        self.stats_fallback = None  # why the engine's collective is not used (all ranks)
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
                self.hgroup = dist.new_group(backend="gloo")
                self._select_stats_path()
            else:
                dist.init_process_group(self.backend)
                self.hgroup = dist.group.WORLD

    def _coll(self, t):
        return t if self.backend == "nccl" else t.cpu()

    def barrier(self):
        if self.world > 1:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.dev.index])
            else:
                dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        t = self._coll(torch.tensor([x], dtype=torch.float64, device=self.dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_ok(self, ok):
        """True iff `ok` holds on every rank (MIN over the host-side gloo
        group: nothing is queued on the device), so every rank takes the
        same branch after it."""
        if self.world == 1:
            return bool(ok)
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.hgroup)
        return int(t.item()) == 1

    def _errors(self, err):
        """Every rank's error text (all_gather_object on the host group)."""
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=self.hgroup)
        return "; ".join(f"rank {r}: {e}" for r, e in enumerate(errs) if e)

    def _try_engine_comm(self):
        """(communicator or None, error text) -- never raises, and bounded:
        rank 0's unique id (or its failure) travels over torch.distributed,
        then every rank calls qe_comm_init_timeout."""
        import ctypes as C
        lib = engine._lib.lib()
        idb = (C.c_uint8 * lib.qe_comm_id_bytes())()
        payload = [None, ""]
        if self.rank == 0:
            try:
                engine.check("qe_comm_unique_id", lib.qe_comm_unique_id(idb))
                payload = [bytes(idb), ""]
            except Exception as e:  # noqa: BLE001 -- every rank learns it below
                payload = [None, f"qe_comm_unique_id: {e}"]
        dist.broadcast_object_list(payload, src=0, group=self.hgroup)
        if payload[0] is None:
            return None, payload[1] if self.rank == 0 else ""
        idb = (C.c_uint8 * len(payload[0])).from_buffer_copy(payload[0])
        comm = C.c_void_p()
        try:
            engine.check("qe_comm_init_timeout", lib.qe_comm_init_timeout(
                C.byref(comm), self.world, self.rank, idb, self.dev.index, COMM_INIT_TIMEOUT_MS))
        except Exception as e:  # noqa: BLE001
            return None, str(e)
        return comm, ""

    def _select_stats_path(self):
        comm, err = self._try_engine_comm()
        if self.all_ok(comm is not None):
            self.comm = comm
            self.stats_path = "qe_allreduce_stats (RCCL)"
            return
        if comm is not None:  # this rank joined, another did not: nobody uses it
            engine._lib.lib().qe_comm_abort(comm)
        self.stats_fallback = self._errors(err) or "engine communicator unavailable"
        self.stats_path = f"torch.distributed all_reduce (FALLBACK: {self.stats_fallback})"

    def _torch_sum(self, folded, host=False):
        """torch's all-reduce of the counters: RCCL on the device, or (host
        = True, the fallback after an engine failure) gloo on a host copy."""
        if self.backend == "nccl" and not host:
            dist.all_reduce(folded, op=dist.ReduceOp.SUM)
            return folded
        t = folded.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.hgroup)
        return t.to(self.dev)

    def _engine_sum(self, folded):
        """qe_allreduce_stats on a stream of its own (after the launch
        stream's work on `folded`) -> error text ("" = enqueued)."""
        import ctypes as C
        gpu = self.dev.type == "cuda"  # (CPU: the rank-logic tests' fake library)
        if gpu:
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(self.dev)
            self._side.wait_stream(torch.cuda.current_stream(self.dev))
        self._done = None
        try:
            engine.check("qe_allreduce_stats", engine._lib.lib().qe_allreduce_stats(
                engine._ptr(folded), folded.numel(), self.comm,
                C.c_void_p(self._side.cuda_stream) if gpu else None))
        except Exception as e:  # noqa: BLE001
            return f"qe_allreduce_stats: {e}"
        if gpu:
            self._done = torch.cuda.Event()
            self._done.record(self._side)
        return ""

    def _engine_wait(self):
        """Wait for the engine all-reduce with a deadline (polling its event,
        never blocking on it) -> error text."""
        t0 = time.monotonic()
        while self._done is not None and not self._done.query():
            if time.monotonic() - t0 > STATS_WAIT_S:
                return f"qe_allreduce_stats did not complete in {STATS_WAIT_S:.0f} s"
            time.sleep(0.001)
        return ""

    def sum_stats(self, folded):
        """All-reduce (sum) of the uint64 statistics vector: RCCL over xGMI
        through qe_allreduce_stats (128 B, once per workload, latency-bound
        and off the data path); gloo rehearsal: torch on the host.  The
        ranks agree on the outcome of every engine all-reduce before using
        it; a failure anywhere aborts the engine communicator on every rank
        (a collective a peer never entered cannot complete) and all of them
        continue on torch's all_reduce, as a reported fallback."""
        if self.world == 1:
            return folded
        if self.comm is None:
            if self.stats_path is None:  # the gloo rehearsal (no engine communicator)
                self.stats_path = f"torch.distributed {self.backend} (rehearsal)"
            return self._torch_sum(folded)
        keep = folded.clone()
        err = self._engine_sum(folded)
        # agreement 1 (host): every rank enqueued it; agreement 2: every rank
        # saw it complete in time.  Either failing aborts the communicator on
        # every rank (a rank whose collective waits for a peer that never
        # enqueued it is released), and the counters go over the host group.
        if self.all_ok(not err):
            err = self._engine_wait()
            if self.all_ok(not err):
                if self._done is not None:
                    torch.cuda.current_stream(self.dev).wait_stream(self._side)
                return folded
        engine._lib.lib().qe_comm_abort(self.comm)
        self.comm = None
        self.stats_fallback = self._errors(err) or "qe_allreduce_stats failed on a rank"
        self.stats_path = f"torch.distributed gloo all_reduce (FALLBACK: {self.stats_fallback})"
        return self._torch_sum(keep, host=True)

    def close(self):
        if self.comm is not None:
            engine._lib.lib().qe_comm_destroy(self.comm)
            self.comm = None
        if self.world > 1:
            dist.destroy_process_group()


# ---------------------------------------------------------------------------
# counter-based synthetic state: every value is a pure function of (seed,
# GLOBAL group id, slot) through the engine's own generator (qe_gen_groups,
# dist 1 = uniform 63-bit), so a rank's shard of a multi-rank run holds
# exactly the groups a single process would hold at the same global ids
# ---------------------------------------------------------------------------
def counter_rows(G, S, seed, goff, dev, stride=None):
    """[S][stride] int64 tensor of 63-bit uniforms keyed by (seed, goff + g, s)
    (stride None: G rounded up to 64)."""
    b = engine.SlotBatch(G, S, dev, masks=(), votes=False, group_offset=goff, stride=stride)
    engine.gen_groups(b, seed, dist=1, p_absent=0)
    return b.match


def progress_round_state(ps, msgs, seed=0x5EED):
    """The progress_step workload: 4 followers in StateReplicate (RecentActive)
    with 0..F in-flight entries, a 4-term-run leader log, and one round of
    messages -- 70 % MsgAppResp accepts, 10 % rejects, 10 % heartbeat
    responses, 10 % none, no message from the leader's own slot 0.  Round 6:
    Next lies above the in-flight entries, as in every reachable Progress
    (an Inflights entry is the last index of a MsgApp sent, OptimisticUpdate
    moved Next past it); rounds 1-5 drew Next within 4 of Match below them."""
    G, S, F, R = ps.G, ps.S, ps.F, ps.R
    goff, dev, st = ps.group_offset, ps.device, ps.stride
    u = lambda k, s=S: counter_rows(G, s, seed + 0x1000 * k, goff, dev, st)  # noqa: E731
    top = 1 << int(os.environ.get("QE_BENCH_INDEX_BITS", "40"))  # A/B knob only
    base = (1 << 20) + u(1, 1)[:st] % (top - (1 << 20))
    ps.match.copy_(base.repeat(S) + u(2) % 64)
    cnt = (u(4) % (F + 1)).to(torch.int32)
    # the newest in-flight entry is Match + 1 + 8 (count - 1)
    ps.next.copy_(ps.match + 1 + 8 * torch.clamp(cnt.to(torch.int64) - 1, min=0) +
                  (cnt > 0).to(torch.int64) + u(3) % 4)
    ps.peer.copy_(cnt * (1 << 16) + (1 | 8))  # StateReplicate, RecentActive, start 0
    ks = 8 * torch.arange(F, device=dev, dtype=torch.int64).view(1, F)
    for s in range(S):  # ring entry k = Match + 1 + 8k (start 0: the live ones are k < count)
        ps.set_ring_slot(s, ps.match[s * st:(s + 1) * st].view(st, 1) + 1 + ks)
    ps.last_index.copy_(base[:G] + 128)
    ps.term_start.copy_(base[:G])
    ps.first_index.copy_(base[:G] - 64)
    ps.committed.copy_(base[:G])
    ps.self_slot.fill_(0)  # the leader's own Progress is slot 0
    rf = ps.run_first.view(R, st)
    for r in range(R):
        rf[r].copy_(base - 65 + 40 * r)
    ps.run_term.view(R, st).copy_(
        torch.arange(1, R + 1, device=dev).repeat_interleave(st).view(R, st))
    ps.run_count.fill_(R)
    v = u(5) % 10
    ty = torch.where(v < 7, 1, torch.where(v == 7, 2, torch.where(v == 8, 3, 0)))
    ty.view(S, st)[0] = 0  # no message from the leader itself
    msgs.type.copy_(ty.to(torch.uint8))
    # acks stay within the leader's log: match + [0, 64] <= base + 127 < lastIndex
    msgs.index.copy_(ps.match + u(6) % 65)
    msgs.reject_hint.copy_(ps.match)
    msgs.log_term.copy_(u(7) % 4)


def psend_state(ps, seed=0x5E4D):
    """The progress_send workload: followers in StateReplicate with room in
    their Inflights (start 0..F-1, count 0..F-1), Next a little past the
    newest in-flight entry (round 6; rounds 1-5: a little past Match)."""
    G, S, F = ps.G, ps.S, ps.F
    goff, dev, st = ps.group_offset, ps.device, ps.stride
    u = lambda k, s=S: counter_rows(G, s, seed + 0x1000 * k, goff, dev, st)  # noqa: E731
    base = (1 << 20) + u(1, 1)[:st] % ((1 << 40) - (1 << 20))
    ps.match.copy_(base.repeat(S) + u(2) % 64)
    start = (u(4) % F).to(torch.int32)
    cnt = (u(5) % F).to(torch.int32)
    ps.next.copy_(ps.match + 1 + cnt.to(torch.int64) + u(3) % 4)  # past Match + count
    ps.peer.copy_(cnt * (1 << 16) + start * (1 << 8) + (1 | 8))  # Replicate, RecentActive
    # in-flight entries in ring order: the entry at position (start + j) % F
    # is Match + 1 + j (the live ones j < count lie just above Match)
    k = torch.arange(F, device=dev, dtype=torch.int64).view(1, F)
    for s in range(S):
        r = slice(s * st, (s + 1) * st)
        j = torch.remainder(k - start[r].view(st, 1).to(torch.int64), F)
        ps.set_ring_slot(s, ps.match[r].view(st, 1) + 1 + j)
    ps.last_index.copy_(base[:G] + 128)
    ps.first_index.copy_(base[:G] - 64)


# ---------------------------------------------------------------------------
# workload setup: returns (step_fn, bytes_per_unit, units_per_step, unit_name)
# ---------------------------------------------------------------------------
def joint_confstates(goff, n, dev, seed=0x5EED):
    """ConfState CSR lists (raft.proto:115-130) of the config-3 shape for the
    global group ids goff .. goff+n-1: Voters[0] = 5 voters, Voters[1] = 5
    voters overlapping Voters[0] in o = 0..5 of them (uniform per group),
    the o peers outside the union are learners -- S = 10 peers per group.
    Peer IDs are gid * 16 + 1 + ((role + r) % 10) with a per-group rotation
    r, so ascending-ID slot order interleaves the halves differently from
    group to group.  (o, r) come from the engine's counter generator keyed
    by the global group id; the lists are built on `dev` and copied to host
    memory, where the packer reads them.  Returns (ConfStates, overlap)."""
    from etcd_amd.packing import ConfStates
    h = counter_rows(n, 1, seed, goff, dev)[:n]
    o = h % 6
    r = (h >> 8) % 10
    base = (torch.arange(goff, goff + n, device=dev, dtype=torch.int64) * 16 + 1).view(n, 1)
    k = torch.arange(10, device=dev)
    rot = (k.view(1, 10) + k.view(10, 1)) % 10                     # rot[r][role]
    outt = torch.stack([rot[:, 5 - ov:10 - ov] for ov in range(6)])  # [o][r][5]
    lrn = torch.stack([(10 - ov + torch.arange(5, device=dev).view(1, 5) + k.view(10, 1)) % 10
                       for ov in range(6)])                         # [o][r][5]
    voters = (base + rot[r, :5]).reshape(-1)
    outgoing = (base + outt[o, r]).reshape(-1)
    learners = torch.masked_select(base + lrn[o, r], torch.arange(5, device=dev).view(1, 5) <
                                   o.view(n, 1))
    loff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    loff[1:] = torch.cumsum(o, 0)
    off5 = torch.arange(n + 1, dtype=torch.int64, device=dev) * 5
    host = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
    cs = ConfStates.from_csr(n, (host(voters), host(off5)), (host(outgoing), host(off5)),
                             (host(learners), host(loff)))
    return cs, o.cpu().numpy()


def pack_joint_batches(b, goff, chunk=1 << 24):
    """Build batch `b`'s masks through the product packer: per 16M-group
    batch, ConfStates -> qe_pack_order (shape bucketing) -> qe_pack_confstate
    with that order -> masks copied into HBM at the batch's positions.
    Returns the device perm (packed position -> global group id - goff)."""
    import ctypes as C
    from etcd_amd import _lib
    from etcd_amd.packing import _np_ptr
    lib = _lib.lib()
    G, S = b.G, b.S
    perm_all = torch.empty(G, dtype=torch.int64, device=b.device)
    md = np.uint16
    for c0 in range(0, G, chunk):
        n = min(chunk, G - c0)
        cs, _ = joint_confstates(goff + c0, n, b.device)
        perm = np.zeros(n, np.uint64)
        nsh = C.c_uint64(0)
        st = cs.struct()
        engine.check("qe_pack_order", lib.qe_pack_order(C.byref(st), S, _np_ptr(perm),
                                                         C.byref(nsh)))
        cs.perm = perm
        st = cs.struct()
        inc, out, lrn = (np.zeros(n, md) for _ in range(3))
        ids = np.empty(S * n, np.uint64)
        nflag = C.c_uint64(0)
        engine.check("qe_pack_confstate", lib.qe_pack_confstate(
            C.byref(st), S, _np_ptr(inc), _np_ptr(out), _np_ptr(lrn), _np_ptr(ids), None,
            C.byref(nflag)))
        assert nflag.value == 0
        for dst, a in ((b.inc, inc), (b.out, out), (b.learner, lrn)):
            dst[c0:c0 + n].copy_(torch.from_numpy(a.view(np.int16)))
        perm_all[c0:c0 + n].copy_(torch.from_numpy((perm + np.uint64(c0)).view(np.int64)))
        del cs, ids
    return perm_all


def setup(name, G, S, kind, d, stats):
    goff = d.rank * G
    if kind in ("majority", "joint", "joint_rot", "joint_packed"):
        masks = () if kind == "majority" else ("inc", "out", "learner")
        b = engine.SlotBatch(G, S, d.dev, masks=masks, group_offset=goff)
        if kind == "joint":
            engine.gen_groups(b, 0x5EED, n_inc=5, n_out=5, mask_mode=2)
        elif kind == "joint_rot":
            engine.gen_groups(b, 0x5EED, n_inc=5, n_out=5, mask_mode=0)
        elif kind == "joint_packed":
            # masks through the packer; Match / votes from the generator at
            # the packed positions (values do not depend on the layout)
            pack_joint_batches(b, goff)
            engine.gen_groups(b, 0x5EED, values_only=True)
        else:
            engine.gen_groups(b, 0x5EED)
        # BASELINE config 2/3 outputs: CommittedIndex + VoteResult per group
        # (8 + 1 B written); TallyVotes granted/rejected are
        # still computed and summed into the statistics counters.
        out = engine.Outputs(G, d.dev, tally=False)
        gs = b.struct()
        os_ = out.struct(stats)
        import ctypes as C
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)

        def step():
            engine.check("qe_commit_vote", lib.qe_commit_vote(C.byref(gs), C.byref(os_), stream))

        # algorithmic bytes per group: every input read once, every output
        # written once: 8S + 2 + 9 = 51 B at S=5
        bpg = b.bytes_per_group(with_outputs=True)
        if kind != "majority":
            # config 3 counts only the union slots' Match: 19 + 8u
            inc = b.inc.to(torch.int32)
            uni = (inc | b.out.to(torch.int32))
            u = torch.zeros(G, dtype=torch.int64, device=d.dev)
            for s in range(S):
                u += (uni >> s) & 1
            mean_u = float(u.double().mean().item())
            bpg = 3 * 2 + 2 * 2 + 8 * mean_u + 9
        return step, bpg, G, "group-evals", {"batch": b, "out": out}
    if kind in ("repl", "repl_joint"):
        joint = kind == "repl_joint"
        b = engine.SlotBatch(G, S, d.dev, masks=("inc", "out") if joint else (), votes=False,
                             group_offset=goff)
        engine.gen_groups(b, 0x5EED, p_absent=0)
        if joint:  # the joint configuration of a one-voter replacement (EnterJoint)
            b.inc.fill_(0b101111)
            b.out.fill_(0b011111)
        rows = b.match_rows()
        lo = rows.min(dim=0).values
        hi = rows.max(dim=0).values
        st = engine.ReplicationState(b, lo.clone(), lo + (hi - lo) // 2, hi + 1024)
        # responses: followers ack a bit beyond their match (pre-generated,
        # resident in HBM).  The kernel writes Match/Next/committed only
        # where they change (as MaybeUpdate / commitTo do), so a re-applied
        # batch would be cheaper than a fresh one: every timed launch starts
        # from the same pristine state (restored outside its HIP events).
        rb = engine.SlotBatch(G, S, d.dev, masks=(), votes=False, group_offset=goff)
        engine.gen_groups(rb, 0xACC, p_absent=0)
        resp = b.match.clone() + (rb.match & 1023)
        del rb
        full = (1 << S) - 1
        rm = torch.full((G,), full & ~1, dtype=torch.uint8, device=d.dev)  # every follower
        acks = torch.full((G,), 0b00111, dtype=torch.uint8, device=d.dev)
        read_ok = torch.empty(G, dtype=torch.uint8, device=d.dev)
        import ctypes as C
        s_ = st.struct()
        m_ = engine.QeReplMsgs(engine._ptr(resp), engine._ptr(rm), engine._ptr(acks),
                               engine._ptr(read_ok), None)
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            engine.check("qe_replication_round",
                         lib.qe_replication_round(C.byref(s_), C.byref(m_), sp, stream))

        pristine = {"match": b.match.clone(), "next": st.next.clone(),
                    "committed": st.committed.clone()}

        def prepare():
            b.match.copy_(pristine["match"])
            st.next.copy_(pristine["next"])
            st.committed.copy_(pristine["committed"])

        # Algorithmic bytes of this round (what the state machine must read
        # and write, once): the responder and ReadIndex-ack masks (2 B),
        # termStart / lastIndex / committed (24 B), every voter's Match (8S),
        # a responder's m.Index and Next (16 B each); writes only where
        # MaybeUpdate / commitTo change a word (as the reference assigns),
        # plus the ReadIndex result byte.  SURVEY.md §8(d)'s 40n + 26 B
        # counts every Next/resp read and every store; this round needs less.
        with torch.no_grad():
            nresp = bin(int(rm[0].item())).count("1")  # every group: same mask
            step()
            torch.cuda.synchronize(d.dev)
            m1 = b.match.view(S, b.stride)[:, :G]
            n1 = st.next.view(S, b.stride)[:, :G]
            m0 = pristine["match"].view(S, b.stride)[:, :G]
            n0 = pristine["next"].view(S, b.stride)[:, :G]
            writes = 8 * (int((m1 != m0).sum()) + int((n1 != n0).sum()) +
                          int((st.committed != pristine["committed"]).sum())) + G
            prepare()
        bpg = 2 + 24 + 8 * S + 16 * nresp + writes / G + (2 if joint else 0)  # + inc/out masks
        return step, bpg, G, "group-rounds", {"b": b, "st": st, "resp": resp,
                                               "prepare": prepare}
    if kind in ("elec", "elec_pvcq"):
        # config 5; elec_pvcq: raft.Config{PreVote, CheckQuorum} with each
        # peer heard from within an election timeout with p = 0.7
        flags = 0 if kind == "elec" else (engine._lib.QE_ELEC_PREVOTE |
                                          engine._lib.QE_ELEC_CHECK_QUORUM)
        p_active = 0 if kind == "elec" else 45875
        b = engine.SlotBatch(G, S, d.dev, masks=("inc",), votes=False, group_offset=goff)
        engine.gen_groups(b, 0x5EED)
        est = engine.ElectionState(b, engine.first_voter_slot(b))
        steps_per_launch = 64
        counter = {"step0": 0}
        import ctypes as C
        s_ = est.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            p = engine.QeElectionParams(0xE1EC, counter["step0"], steps_per_launch, 13107, 32768,
                                        flags, p_active, 0, None, None, None, 0)
            engine.check("qe_election_steps", lib.qe_election_steps(C.byref(s_), C.byref(p), sp, stream))
            counter["step0"] += steps_per_launch

        # HBM bytes per group-step: state in+out / steps (register-resident)
        bpg = (8 + 1 + 1 + 1 + 1 + 1 + 8 + 1 + 1 + 1) / steps_per_launch
        return step, bpg, G * steps_per_launch, "group-steps", {"b": b, "est": est}
    if kind in ("progress", "progress_joint"):
        F, R, ME = 8, int(os.environ.get("QE_BENCH_RUNS", "4")), 16  # R: A/B knob only
        joint = kind == "progress_joint"
        ps = engine.ProgressState(G, S, F, R, d.dev, group_offset=goff, extras=("self_slot",),
                                  max_ents=ME, masks=("inc", "out") if joint else (),
                                  ring16=RING16 and R <= 4)
        if joint:  # EnterJoint of a one-voter replacement, as config4_repl_joint
            ps.inc.fill_(0b101111)
            ps.out.fill_(0b011111)
        msgs = engine.PeerMsgs(ps)
        msgs.snap = msgs.timeout_now = None  # no snapshots / transfers in this workload
        # no ReadIndex in this workload (heartbeat rounds carry it); the
        # round-3 output set, so the figures stay comparable
        msgs.read_released = msgs.term_commit = msgs.term_commit_index = None
        progress_round_state(ps, msgs)
        # Every timed launch steps the SAME fresh state with the same round
        # of messages: the mutable state is restored from a pristine copy
        # before each launch (outside the kernel's HIP events), so no launch
        # sees stale, already-applied duplicates.  The 32-bit rings need no
        # restore: a round writes free positions (live ones are written back
        # unchanged), and the live entries it reads are the restored (start,
        # count) window; the 16-bit form's offsets are re-based on the new
        # Next, so those are restored too.
        mutable = ("match", "next", "pending", "peer", "committed") + (
            ("infl16",) if ps.infl16 is not None else ())
        pristine = {k: getattr(ps, k).clone() for k in mutable}

        def prepare():
            for k in mutable:
                getattr(ps, k).copy_(pristine[k])

        # Algorithmic bytes of this round: the instrumented kernel variant
        # counts every field the state machine reads or writes (reads of the
        # message, the Progress fields each event needs, PendingSnapshot only
        # in StateSnapshot, the Inflights entries FreeLE examines, the
        # term-run table when findConflictByTerm runs; writes of changed
        # fields, appended Inflights entries and the outputs), once each --
        # the rules the oracle restates (tests/test_gpu_progress.py checks
        # the two counts are equal on this workload's state).
        prepare()
        total = engine.progress_bytes_requested(ps, msgs)
        prepare()
        bpg = total / G
        import ctypes as C
        p_, m_ = ps.struct(), msgs.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            engine.check("qe_progress_step",
                         lib.qe_progress_step(C.byref(p_), C.byref(m_), sp, stream))

        return step, bpg, G, "group-rounds", {"ps": ps, "msgs": msgs, "prepare": prepare}
    if kind == "propose":
        # stepLeader MsgProp -> appendEntry -> bcastAppend (raft/raft.go:
        # 1019-1076, :621-642, :515-522) on the progress_send state, the
        # leader in slot 0; every group proposes 3 entries each launch
        F = 8
        ps = engine.ProgressState(G, S, F, 1, d.dev, group_offset=goff, extras=("self_slot",),
                                  max_ents=0, ring16=RING16)
        psend_state(ps)
        ps.self_slot.fill_(0)
        ps.term_start.copy_(ps.last_index)  # the leader's term started at its last entry
        pr = engine.Proposals(ps, max_uncommitted=1 << 30)
        pr.num_entries.fill_(3)
        pr.payload.fill_(24)
        pr.uncommitted_size.fill_(100)
        mutable = ("match", "next", "peer", "committed", "last_index") + (
            ("infl16",) if RING16 else ())
        pristine = {k: getattr(ps, k).clone() for k in mutable}
        unc0 = pr.uncommitted_size.clone()

        def prepare():
            for k in mutable:
                getattr(ps, k).copy_(pristine[k])
            pr.uncommitted_size.copy_(unc0)

        # algorithmic bytes: the instrumented variant counts every field
        # the reference logic reads or writes once (the
        # oracle's count is equal, tests/test_gpu_propose.py)
        prepare()
        bpg = engine.propose_bytes_requested(ps, pr) / G
        prepare()
        import ctypes as C
        p_, q_ = ps.struct(), pr.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            engine.check("qe_propose", lib.qe_propose(C.byref(p_), C.byref(q_), sp, stream))

        def verify():
            return bool((pr.result == 1).all())

        return step, bpg, G, "group-proposals", {"ps": ps, "pr": pr, "prepare": prepare,
                                                 "verify": verify}

    if kind == "switch":
        # raft.switchToConfig (raft/raft.go:1651-1700) on the progress_send
        # state: maybeCommit under the new quorum, bcastAppend or the probe of
        # every peer, abortLeaderTransfer
        F = 8
        ps = engine.ProgressState(G, S, F, 1, d.dev, group_offset=goff, masks=("inc",),
                                  extras=("self_slot", "tracked", "lead_transferee"), max_ents=0,
                                  ring16=RING16)
        psend_state(ps)
        st = ps.stride
        li = ps.last_index[:G]
        ps.self_slot.fill_(0)
        ps.match[:G].copy_(li)  # the leader's own Progress: Match = lastIndex
        ps.next[:G].copy_(li + 1)
        ps.term_start.copy_(li - 127)  # the leader's term holds the followers' acks
        h = counter_rows(G, 1, 0x5C0F, goff, d.dev)[:G]
        remove = (h & 1) == 1
        ps.inc.copy_(torch.where(remove, 0b00111, 0b11111).to(torch.uint8))
        ps.tracked.copy_(torch.where(remove, 0b10111, 0b11111).to(torch.uint8))
        ps.lead_transferee.copy_(torch.where(((h >> 1) & 7) == 0, 3, 0xFF).to(torch.uint8))
        m = ps.match.view(S, st)[:4, :G]
        ps.committed.copy_(m.sort(dim=0, descending=True).values[2])  # the old quorum's
        sw = engine.Switch(ps)
        mutable = ("next", "peer", "committed", "lead_transferee") + (("infl16",) if RING16 else ())
        pristine = {k: getattr(ps, k).clone() for k in mutable}

        def prepare():
            for k in mutable:
                getattr(ps, k).copy_(pristine[k])

        # algorithmic bytes: the instrumented variant counts every field the
        # reference logic reads or writes once (the oracle's
        # count is equal, tests/test_gpu_switch.py)
        prepare()
        bpg = engine.switch_bytes_requested(ps, sw) / G
        prepare()
        import ctypes as C
        p_, q_ = ps.struct(), sw.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            engine.check("qe_switch_config", lib.qe_switch_config(C.byref(p_), C.byref(q_), sp,
                                                                   stream))

        def verify():
            out = sw.result & engine._lib.QE_SW_OUTCOME
            return bool(((out == engine._lib.QE_SW_BCAST) | (out == engine._lib.QE_SW_PROBE)).all())

        return step, bpg, G, "group-switches", {"ps": ps, "sw": sw, "prepare": prepare,
                                                "verify": verify}

    if kind == "heartbeat":
        # stepLeader MsgBeat -> bcastHeartbeat -> sendHeartbeat (raft/raft.go:
        # 524-541, :494-510): per follower min(Match, committed), the context
        # of the last pending ReadIndex request (lastPendingRequestCtx)
        ps = engine.ProgressState(G, S, 8, 1, d.dev, group_offset=goff,
                                  extras=("self_slot", "reads"), max_ents=0, ring16=RING16)
        psend_state(ps)
        ps.self_slot.fill_(0)
        ps.committed.copy_(ps.last_index[:G] - 32)
        qn = counter_rows(G, 1, 0x4EAD, goff, d.dev)[:G] % (engine._lib.QE_READ_QUEUE + 1)
        ps.read_count.copy_(qn.to(torch.uint8))
        commit = torch.zeros(S * ps.stride, dtype=torch.int64, device=d.dev)
        ctx = torch.zeros(G, dtype=torch.int32, device=d.dev)
        sent = torch.zeros(G, dtype=torch.uint8, device=d.dev)
        # algorithmic bytes per group: self slot 1, committed 8, the queue's
        # count 1 and head 4, the context 4 and the sent mask 1 written, and
        # per follower sent to (4) its Match read and its Commit written
        bpg = 1 + 8 + 1 + 4 + 4 + 1 + (S - 1) * 16
        import ctypes as C
        p_ = ps.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        cp, xp, sp_ = engine._ptr(commit), engine._ptr(ctx), engine._ptr(sent)

        def step():
            engine.check("qe_heartbeat", lib.qe_heartbeat(C.byref(p_), cp, xp, sp_, stream))

        def verify():
            full = (1 << S) - 2
            m = ps.match.view(S, -1)[1:, :G]
            c = commit.view(S, -1)[1:, :G]
            want = torch.minimum(m, ps.committed[:G].view(1, G))
            qh = ps.read_head[:G].to(torch.int64)
            cx = torch.where(qn > 0, qh + qn - 1, torch.zeros_like(qn))
            return (bool((sent.to(torch.int32) == full).all()) and bool((c == want).all())
                    and bool((ctx.to(torch.int64) & 0xFFFFFFFF == cx).all()))

        return step, bpg, G, "group-heartbeats", {"ps": ps, "commit": commit, "ctx": ctx,
                                                  "sent": sent, "verify": verify}

    if kind == "psend":
        # raft.appendEntry -> bcastAppend (raft/raft.go:515-522, :432-492):
        # every follower in StateReplicate with room in its Inflights gets one
        # MsgApp of up to 16 entries (one ring append, OptimisticUpdate)
        F, ME = 8, 16
        ps = engine.ProgressState(G, S, F, 1, d.dev, group_offset=goff, max_ents=ME, ring16=RING16)
        psend_state(ps)
        full = (1 << S) - 1
        want = torch.full((G,), full & ~1, dtype=torch.uint8, device=d.dev)  # not the leader
        sent = torch.zeros(G, dtype=torch.uint8, device=d.dev)
        snap = torch.zeros(G, dtype=torch.uint8, device=d.dev)
        mutable = ("next", "peer") + (("infl16",) if RING16 else ())
        pristine = {k: getattr(ps, k).clone() for k in mutable}

        def prepare():
            for k in mutable:
                getattr(ps, k).copy_(pristine[k])

        import ctypes as C
        p_ = ps.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)

        def step():
            engine.check("qe_progress_send", lib.qe_progress_send(
                C.byref(p_), engine._ptr(want), 0, engine._ptr(sent), engine._ptr(snap), stream))

        # per group: want mask, firstIndex/lastIndex read, sent/snap masks
        # written; per wanted peer Next and the packed word read, Next, the
        # word (count changes) and the appended entry written -- its 32-bit
        # word (ABI 4) or 16-bit offset (ABI 8): 1 + 16 + 2 + 4 * (12 + 16) =
        # 131 B, or 123 B
        nw = bin(full & ~1).count("1")
        bpg = 1 + 16 + 2 + nw * (12 + 12 + (2 if RING16 else 4))
        return step, bpg, G, "group-bcasts", {"ps": ps, "prepare": prepare,
                                              "t": (want, sent, snap)}
    if kind == "cq":
        ps = engine.ProgressState(G, S, 1, 1, d.dev, group_offset=goff, extras=("self_slot",))
        act = counter_rows(G, S, 0xC4EC, goff, d.dev, ps.stride) % 10 < 7  # heard from within the timeout
        ps.peer.copy_(act.to(torch.int32) * 8 + 1)  # StateReplicate (+ RecentActive)
        ps.self_slot.fill_(0)
        del act
        qa = torch.empty(G, dtype=torch.uint8, device=d.dev)
        pristine = ps.peer.clone()

        def prepare():
            ps.peer.copy_(pristine)

        import ctypes as C
        p_ = ps.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)
        sp = engine._ptr(stats)

        def step():
            engine.check("qe_check_quorum", lib.qe_check_quorum(C.byref(p_), engine._ptr(qa), sp,
                                                                  stream))

        # per group: self_slot read and the quorum-active byte written; every
        # slot's word read (all tracked) and the words whose RecentActive
        # changes written (counted on this state)
        step()
        torch.cuda.synchronize(d.dev)
        changed = int((ps.peer.view(S, ps.stride)[:, :G] != pristine.view(S, ps.stride)[:, :G]).sum())
        prepare()
        bpg = 1 + 4 * S + 1 + 4 * changed / G
        return step, bpg, G, "group-checks", {"ps": ps, "prepare": prepare, "t": qa}
    if kind == "collect":
        gen = torch.Generator(device=d.dev).manual_seed(0xC011 + d.rank)
        flags = (torch.rand(G, device=d.dev, generator=gen) < 0.5).to(torch.uint8)
        values = torch.randint(0, 1 << 40, (G,), device=d.dev, generator=gen)
        import ctypes as C
        lib = engine._lib.lib()
        scratch = torch.empty((lib.qe_collect_scratch_bytes(G) + 7) // 8, dtype=torch.int64,
                              device=d.dev)
        groups = torch.empty(G, dtype=torch.int64, device=d.dev)
        vals = torch.empty(G, dtype=torch.int64, device=d.dev)
        count = torch.empty(1, dtype=torch.int64, device=d.dev)
        stream = engine._stream(d.dev)
        args_ = [G, goff, None] + [engine._ptr(t) for t in (flags, values, groups, vals, count,
                                                             scratch)]

        def step():
            engine.check("qe_collect", lib.qe_collect(*args_, stream))

        step()
        torch.cuda.synchronize(d.dev)
        sel = int(count.item())
        # every flag read once; per selected group its value read and the id
        # and value written (8 + 16 B)
        bpg = 1 + 24 * sel / G
        return step, bpg, G, "groups", {"t": (flags, values, scratch, groups, vals, count)}
    if kind == "confchange":
        cs = engine.ConfState(G, S, d.dev)
        ps = engine.ProgressState(G, S, 1, 1, d.dev)
        ch = engine.ConfChanges(G, S, 2, d.dev)
        gid = torch.arange(G, device=d.dev, dtype=torch.int64) + goff
        ids = gid.view(1, G) * 8 + torch.arange(1, S + 1, device=d.dev).view(S, 1)  # [S][G]
        ids[4] = 0  # slot 4 free
        cs.slot_ids.copy_(ids.reshape(-1))
        cs.inc.fill_(0b00111)
        cs.learner.fill_(0b01000)
        cs.is_learner.fill_(0b01000)
        cs.tracked.fill_(0b01111)
        ch.op.fill_(1)  # QE_CC_OP_SIMPLE
        ch.count.fill_(2)
        ch.type.view(2, G)[0].fill_(0)  # AddNode(learner in slot 3): promote
        ch.type.view(2, G)[1].fill_(3)  # AddLearnerNode(new id)
        ch.node_id.view(2, G)[0].copy_(gid * 8 + 4)
        ch.node_id.view(2, G)[1].copy_(gid * 8 + 7)
        ch.last_index.copy_(gid + 100)
        mutable = ("slot_ids", "inc", "out", "learner", "learners_next", "is_learner",
                   "tracked", "auto_leave")
        pristine = {k: getattr(cs, k).clone() for k in mutable}

        def prepare():
            for k in mutable:
                getattr(cs, k).copy_(pristine[k])

        # every input read once (op, count, 2 changes, last_index, 6 masks,
        # auto_leave, the 4 tracked slots' ids) plus the outputs and the words
        # the change rewrites, once (result, new_progress; inc, learner,
        # is_learner and tracked change, out / learners_next / auto_leave do
        # not; one slot ID -- its own [S][G] row, ABI 3; one initialised
        # Progress row: match/next/pending + the packed word).
        bpg = (1 + 1 + 2 * 9 + 8 + 6 + 1 + 8 * 4) + (1 + 1 + 4 + 8 + 28)
        import ctypes as C
        c_, x_, p_ = cs.struct(), ch.struct(), ps.struct()
        lib = engine._lib.lib()
        stream = engine._stream(d.dev)

        def step():
            engine.check("qe_confchange",
                         lib.qe_confchange(C.byref(c_), C.byref(x_), C.byref(p_), stream))

        def verify():
            ok = bool((ch.result == 0).all()) and bool((cs.inc == 0b01111).all())
            return ok and bool((cs.learner == 0b10000).all())

        return step, bpg, G, "group-changes", {"cs": cs, "ps": ps, "ch": ch,
                                               "prepare": prepare, "verify": verify}
    raise ValueError(kind)


def time_steps(step, d, steps, warmup, prepare=None):
    for _ in range(warmup):
        if prepare:
            prepare()
        step()
    d.barrier()
    torch.cuda.synchronize(d.dev)
    stream = torch.cuda.current_stream(d.dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in evs:
        if prepare:
            prepare()
        a.record(stream)
        step()
        b.record(stream)
    d.barrier()
    torch.cuda.synchronize(d.dev)
    wall = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    return wall, kern_ms


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(args, S=5):
    """Oracle port timed on this host's cores over a bounded sample."""
    from oracle import orc
    G = args.cpu_groups
    threads = args.cpu_threads or cpu_share()
    hb = orc.Batch(G, S, masks=())
    orc.gen_batch(hb, 0x5EED, threads=threads)
    commit = np.zeros(G, np.uint64)
    vote = np.zeros(G, np.uint8)
    L = orc.lib()
    w = L.orc_gf_build(G, S, G, orc.P(hb.match), None, None, None, orc.P(hb.voted),
                       orc.P(hb.granted))
    try:
        L.orc_gf_run(w, orc.P(commit), orc.P(vote), 1, threads)  # warm-up
        t1 = L.orc_gf_run(w, orc.P(commit), orc.P(vote), 1, threads)
        reps = max(1, int(10.0 / max(t1, 1e-6)))
        t = L.orc_gf_run(w, orc.P(commit), orc.P(vote), reps, threads)
        gf_rate = G * reps / t
        # one thread, for the per-core rate and the scaling over the share
        t1s = L.orc_gf_run(w, orc.P(commit), orc.P(vote), 1, 1)
        reps1 = max(1, int(3.0 / max(t1s, 1e-6)))
        gf_rate1 = G * reps1 / L.orc_gf_run(w, orc.P(commit), orc.P(vote), reps1, 1)
    finally:
        L.orc_gf_free(w)
    # the SoA restatement (strongest CPU variant)
    L.orc_soa_run(G, S, G, orc.P(hb.match), None, None, orc.P(hb.voted), orc.P(hb.granted),
                  orc.P(commit), orc.P(vote), 1, threads)
    t1 = L.orc_soa_run(G, S, G, orc.P(hb.match), None, None, orc.P(hb.voted), orc.P(hb.granted),
                       orc.P(commit), orc.P(vote), 1, threads)
    reps2 = max(1, int(3.0 / max(t1, 1e-6)))
    t2 = L.orc_soa_run(G, S, G, orc.P(hb.match), None, None, orc.P(hb.voted), orc.P(hb.granted),
                       orc.P(commit), orc.P(vote), reps2, threads)
    soa_rate = G * reps2 / t2
    host_cpus = os.cpu_count()
    return {
        "value": gf_rate, "unit": "group-evals/s", "cores": threads, "kind": "port",
        "sample": (f"{G} groups x 5 voters x {reps} passes (~10 s): Go-faithful map/AckedIndexer "
                   f"loop (oracle/quorum_oracle.c orc_gf_run, CommittedIndex+VoteResult per "
                   f"group), OpenMP {threads} threads = this process's CPU share "
                   f"(affinity {len(os.sched_getaffinity(0))} CPUs, OMP_NUM_THREADS "
                   f"{os.environ.get('OMP_NUM_THREADS', 'unset')}) of a {host_cpus}-CPU "
                   f"{cpu_model()} host"),
        "cpu_model": cpu_model(), "host_cpus": host_cpus,
        "one_thread_value": gf_rate1,
        "scaling_efficiency": gf_rate / (gf_rate1 * threads),
        # the north star quotes the Go loop over the host's own cores; this
        # box grants the process a CPU share (OMP_NUM_THREADS), so the whole
        # host is not run here: the per-thread rate measured at the share,
        # times every host CPU, is an upper bound (scaling is at most linear)
        "full_host_value": gf_rate / threads * host_cpus,
        "full_host_basis": (f"ESTIMATE, not measured: the {threads}-thread rate / {threads} x "
                            f"{host_cpus} host CPUs (linear scaling, an upper bound; measured "
                            f"scaling 1 -> {threads} threads: "
                            f"{gf_rate / (gf_rate1 * threads):.2f} of linear)"),
        "soa_value": soa_rate,
        "soa_sample": f"{G} groups x {reps2} passes, SoA restatement (orc_soa_run), {threads} threads",
    }


def load_pmc(workload):
    """The committed rocprofv3 PMC record of a workload's dominant kernel
    (profiles/pmc_traffic.json, scripts/summarize_workloads.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {})
    except (OSError, ValueError):
        return {}


def load_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary."""
    return load_pmc(workload).get("hbm_bytes_per_launch")


# Vector-memory instruction cost on MI355X, streaming probe (scripts/
# vmem_probe.hip, tlb_probe.hip; profiles/r02d_vmem_probe.txt): cycles per
# wave instruction per CU at 2.4 GHz -- a u64 row (dwordx2, 64 lanes) ~57
# (HBM-bound when full; >= 42 however few lanes are active), a byte row ~22.5.
VMEM_PROBE_CYC = {"u64_row": 57.0, "u64_row_floor": 42.0, "u8_row": 22.5,
                  "source": "profiles/r02d_vmem_probe.txt"}


def vmem_issue(workload, kern_ms, units):
    """Vector-memory instructions per launch (SQ_INSTS_VMEM_RD + _WR,
    committed PMC) and the cycles each costs a CU at the measured kernel time,
    for comparison with the streaming probe's per-instruction cost."""
    t = load_pmc(workload)
    rd, wr = t.get("vmem_rd_per_launch"), t.get("vmem_wr_per_launch")
    if not rd or wr is None:
        return None
    n = rd + wr
    return {"vmem_insts_per_launch": n, "vmem_rd": rd, "vmem_wr": wr,
            "vmem_per_tile": n / (units / 64.0),
            "cycles_per_vmem_inst_per_cu": kern_ms / 1000.0 * 2.4e9 * 256 / n,
            "probe_cycles": VMEM_PROBE_CYC, "source": t.get("profile")}


def occupancy(workload):
    """Registers, LDS and resident waves per SIMD of the workload's dominant
    kernel(s) (the PMC record's kernel name looked up in
    profiles/kernel_resources.json, scripts/kernel_resources.py)."""
    names = load_pmc(workload).get("kernel")
    try:
        with open(os.path.join(ROOT, "profiles", "kernel_resources.json")) as f:
            res = json.load(f)
    except (OSError, ValueError):
        return None
    if not names:
        return None
    bare = lambda x: x[5:] if x.startswith("void ") else x  # noqa: E731
    res = {bare(k): v for k, v in res.items()}
    out = {}
    for n in names.split(" + "):
        n = bare(n)
        if n not in res:  # a record made before a defaulted template flag was added (ABI 8: N16)
            n = n.replace(">(", ", false>(", 1)
        if n in res:
            out[n[:n.index("(")]] = {k: res[n][k] for k in ("vgpr", "scratch_bytes", "lds_bytes",
                                                            "waves_per_simd")}
    return out or None


def valu_roofline(workload, kern_ms, units):
    """VALU-issue roofline of a VALU-bound kernel: its VALU instructions per
    launch (SQ_INSTS_VALU, committed PMC) over the live kernel time, against
    VALU_PEAK_WIPS."""
    v = load_pmc(workload).get("valu_insts_per_launch")
    if not v:
        return None
    ach = v / (kern_ms / 1000.0)
    out = {"bound": "valu", "achieved": ach, "peak": VALU_PEAK_WIPS,
           "unit": "wave64 VALU instructions/s", "frac": ach / VALU_PEAK_WIPS,
           "valu_insts_per_launch": v, "valu_per_unit": v / units,
           "lane_ops_per_unit": 64 * v / units,
           "source": load_pmc(workload).get("profile")}
    # the SIMD-cycle view (scripts/valu_cost.py): each opcode at its measured
    # issue cost (v_mul_lo_u32 and v_bcnt_u32_b32 take two full-rate slots),
    # over the kernel's own shader cycles in the same PMC pass
    try:
        with open(os.path.join(ROOT, "profiles", "valu_cost.json")) as f:
            vc = json.load(f)["workloads"].get(workload)
    except (OSError, ValueError, KeyError):
        vc = None
    if vc:
        out.update(cycles_frac=vc["cycles_frac"], insts_frac_measured_clock=vc["insts_frac"],
                   avg_cycles_per_inst=vc["avg_cycles_per_inst"],
                   full_rate_cycles_per_inst=vc["full_rate_cycles"],
                   cycles_source="profiles/valu_cost.json")
    return out


def run_workload(name, args, d, steps, warmup):
    desc, G, S, kind = WORKLOADS[name]
    if args.groups and name == args.workload:
        G = args.groups
    elif name != args.workload and args.aux_groups_div > 1:
        G = max(1 << 16, G // args.aux_groups_div)
    stats = engine.stats_buffer(d.dev)
    step, bpu, units, unit_name, keep = setup(name, G, S, kind, d, stats)
    torch.cuda.synchronize(d.dev)
    prepare = keep.get("prepare")
    wall, kern_ms = time_steps(step, d, steps, warmup, prepare)
    if keep.get("verify"):
        torch.cuda.synchronize(d.dev)
        assert keep["verify"](), f"{name}: unexpected result"
    kern_avg = d.max(float(np.mean(kern_ms)))
    # with a per-launch state restore the wall clock also holds the restore
    # copies: the step time is then the launch's own HIP-event time
    ms_step = kern_avg if prepare else d.max(wall * 1000.0 / steps)
    folded = d.sum_stats(engine.stats_reduce(stats))
    st = engine.stats_dict(folded)
    value = units * d.world / (ms_step / 1000.0)
    achieved = bpu * units / (kern_avg / 1000.0) / 1e9
    del keep
    torch.cuda.empty_cache()
    extra = {}
    if kind in ("elec", "elec_pvcq", "progress", "progress_joint"):
        rv = valu_roofline(name, kern_avg, units)
        if rv:
            extra["roofline_valu"] = rv
    vi = vmem_issue(name, kern_avg, units) if kind not in ("elec", "elec_pvcq") else None
    if vi:  # (the elections are VALU-bound: roofline_valu)
        extra["vmem_issue"] = vi
    oc = occupancy(name)
    if oc:
        extra["occupancy"] = oc
    if kind in ("progress", "progress_joint", "propose", "switch", "psend"):
        # the Inflights rings' device form (ABI 8: 16-bit offsets below Next)
        extra["inflights"] = "16-bit (ABI 8)" if RING16 else "32-bit (ABI 4)"
    return {**extra,
        "desc": desc, "groups_per_gpu": G, "slots": S, "units_per_step": units,
        "unit": f"{unit_name}/s", "value": value, "ms_per_step": ms_step,
        "kernel_ms": kern_avg, "bytes_per_unit": bpu,
        "achieved_GBs": achieved, "hbm_frac": achieved / HBM_PEAK_GBS,
        "invariant_violations": st["invariant_violations"], "checksum": st["checksum"],
        "stats": st,
    }


def pcie_inclusive(args, d):
    """The headline evaluation (config 2, 5 voters) with its inputs and
    outputs in pinned HOST memory, as a caller that keeps the Progress maps on
    the host would run it: per step, H2D of Match / voted / granted (42 B per
    group), qe_commit_vote, D2H of commit / vote (9 B per group), all on the
    launch stream.  Not the headline: `value` there is with inputs resident
    in HBM (PCIe-inclusive rate)."""
    G, S, steps = 1 << 24, 5, 10
    b = engine.SlotBatch(G, S, d.dev, masks=(), group_offset=d.rank * G)
    engine.gen_groups(b, 0x5EED)
    out = engine.Outputs(G, d.dev, tally=False)
    pin = lambda t: torch.empty(t.shape, dtype=t.dtype, pin_memory=True)  # noqa: E731
    h_in = [(pin(t), t) for t in (b.match, b.voted, b.granted)]
    for h, t in h_in:
        h.copy_(t)
    h_out = [(pin(t), t) for t in (out.commit, out.vote)]
    import ctypes as C
    gs, os_ = b.struct(), out.struct()
    lib = engine._lib.lib()
    stream = engine._stream(d.dev)

    def step():
        for h, t in h_in:
            t.copy_(h, non_blocking=True)
        engine.check("qe_commit_vote", lib.qe_commit_vote(C.byref(gs), C.byref(os_), stream))
        for h, t in h_out:
            h.copy_(t, non_blocking=True)

    wall, ms = time_steps(step, d, steps, 2)
    ms_step = d.max(float(np.mean(ms)))
    moved = sum(h.numel() * h.element_size() for h, _ in h_in + h_out)
    res = {"desc": "config 2 (16M groups x 5 voters) with inputs/outputs in pinned host memory: "
                   "H2D 42 B + kernel + D2H 9 B per group, one stream",
           "value": G * d.world / (ms_step / 1000.0), "unit": "group-evals/s",
           "ms_per_step": ms_step, "pcie_bytes_per_step": moved,
           "pcie_GBs": moved / (ms_step / 1000.0) / 1e9}
    del h_in, h_out, b, out
    torch.cuda.empty_cache()
    return res


def config1(args, d):
    """BASELINE configs[0]: BenchmarkMajorityConfig_CommittedIndex-style
    (raft/quorum/bench_test.go:24-40) -- 1M groups x 3 voters, values
    rand.Int63-like (generator dist 1), CommittedIndex only.  A 32 MB pass is
    launch-bound, so 100 launches are captured in one hipGraph and replayed.
    The CPU port runs the same 1M x 3 batch (Go-faithful map loop)."""
    G, S, reps = 1 << 20, 3, 100
    b = engine.SlotBatch(G, S, d.dev, masks=(), votes=False, group_offset=d.rank * G)
    engine.gen_groups(b, 0x5EED, dist=1, p_absent=0)
    commit = torch.empty(G, dtype=torch.int64, device=d.dev)
    import ctypes as C
    gs = b.struct()
    lib = engine._lib.lib()
    engine.committed_index(b, commit)  # warm-up (occupancy query, code load)
    torch.cuda.synchronize(d.dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        stream = engine._stream(d.dev)
        for _ in range(reps):
            engine.check("qe_committed_index", lib.qe_committed_index(
                C.byref(gs), engine._ptr(commit), stream))
    for _ in range(3):
        g.replay()
    d.barrier()
    torch.cuda.synchronize(d.dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(5):
        g.replay()
    ev1.record()
    torch.cuda.synchronize(d.dev)
    ms = d.max(ev0.elapsed_time(ev1) / (5 * reps))
    res = {"desc": "1M groups x 3-voter MajorityConfig CommittedIndex (bench_test.go shape), "
                   "hipGraph of 100 launches; 32 MB working set is Infinity-Cache resident, "
                   "so hbm_frac is not an HBM roofline here", "value": G * d.world / (ms / 1000.0),
           "unit": "group-evals/s", "kernel_ms": ms, "bytes_per_unit": 8 * S + 8,
           "achieved_GBs": (8 * S + 8) * G / (ms / 1000.0) / 1e9}
    res["hbm_frac"] = res["achieved_GBs"] / HBM_PEAK_GBS
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        from oracle import orc
        threads = args.cpu_threads or cpu_share()
        hb = orc.Batch(G, S, masks=(), votes=False)
        orc.gen_batch(hb, 0x5EED, dist=1, p_absent=0, threads=threads)
        # CPU result must equal the GPU's (parity at the reference's own shape)
        c_ref = orc.commit_vote(hb)[0]
        assert np.array_equal(commit.cpu().numpy().view(np.uint64), c_ref), "config1 mismatch"
        L = orc.lib()
        cc = np.zeros(G, np.uint64)
        vv = np.zeros(G, np.uint8)
        zero = np.zeros(G, np.uint8)
        w = L.orc_gf_build(G, S, G, orc.P(hb.match), None, None, None, orc.P(zero), orc.P(zero))
        try:
            L.orc_gf_run(w, orc.P(cc), orc.P(vv), 1, threads)
            t1 = L.orc_gf_run(w, orc.P(cc), orc.P(vv), 1, threads)
            n = max(1, int(1.0 / max(t1, 1e-6)))
            t = L.orc_gf_run(w, orc.P(cc), orc.P(vv), n, threads)
        finally:
            L.orc_gf_free(w)
        assert np.array_equal(cc, c_ref)
        res["cpu_port_value"] = G * n / t
        res["cpu_port_cores"] = threads
        res["speedup_vs_cpu_port"] = res["value"] / res["cpu_port_value"]
    del b, commit, g
    torch.cuda.empty_cache()
    return res


def main():
    global engine
    args = parse()
    maybe_spawn(args)  # --gpus N > 1 outside torchrun: relaunch as N ranks (exits)
    from etcd_amd import engine as _engine
    engine = _engine
    d = Dist()
    if d.world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={d.world}", file=sys.stderr)
        sys.exit(2)
    if d.world > 1:
        # the host packer (config3_joint_packed) runs in every rank at once:
        # each gets its share of this process's CPUs, not all of them
        local = int(os.environ.get("LOCAL_WORLD_SIZE", str(d.world)))
        engine._lib.lib().qe_pack_threads(max(1, cpu_share() // max(1, local)))
    main_res = run_workload(args.workload, args, d, args.steps, args.warmup)
    aux = {}
    if not args.no_aux:
        aux["config1_n3"] = config1(args, d)
        aux["config2_n5_pcie"] = pcie_inclusive(args, d)
        for name in WORKLOADS:
            if name == args.workload:
                continue
            r = run_workload(name, args, d, max(5, args.steps // 2), max(2, args.warmup // 2))
            aux[name] = {k: r[k] for k in ("desc", "value", "unit", "kernel_ms", "bytes_per_unit",
                                           "achieved_GBs", "hbm_frac", "invariant_violations")}
            for k in ("roofline_valu", "vmem_issue", "occupancy", "inflights"):
                if k in r:
                    aux[name][k] = r[k]

    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    if d.rank == 0:
        desc, G, S, kind = WORKLOADS[args.workload]
        traffic = load_traffic(args.workload)
        majority_like = kind in ("majority", "joint", "joint_rot", "joint_packed")
        vs = None
        if cpu is not None and majority_like:
            vs = main_res["value"] / cpu["value"]
        line = {
            "metric": METRIC,
            "value": main_res["value"],
            "unit": "group-evals/s" if majority_like else main_res["unit"],
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": vs,
            "vs_baseline_basis": ("value / cpu_baseline.value: the metric's 'speedup vs Go host' "
                                  "against the measured CPU port (BASELINE.md publishes no "
                                  "number); null when no CPU baseline ran (N > 1)"),
            "dtype": "u64",
            "data": "synthetic: counter-based splitmix64 generator, inputs resident in HBM",
            "config": {
                "workload": f"{args.workload}: {desc}",
                "groups_per_gpu": main_res["groups_per_gpu"],
                "global_groups": main_res["groups_per_gpu"] * d.world,
                "voters": S,
                "parallelism": f"group-sharded x{d.world} (no data-path collective; "
                               f"RCCL all-reduce of 16 stats counters after the run)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": main_res["achieved_GBs"],
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": main_res["hbm_frac"],
                "traffic": traffic,
                "kernel": "qe::k_cv_stream" if majority_like else kind,
                "kernel_ms": main_res["kernel_ms"],
                "bytes_per_unit": main_res["bytes_per_unit"],
            },
            "cpu_baseline": cpu,
            "checks": {"invariant_violations": main_res["invariant_violations"],
                       "stats_checksum": main_res["checksum"],
                       "stats_allreduce": None if d.world == 1 else d.stats_path,
                       "stats_fallback": d.stats_fallback},
            "aux": aux,
        }
        print(json.dumps(line))
    fallback = d.stats_fallback
    d.close()
    sys.exit(exit_status(fallback, args.allow_stats_fallback))


def exit_status(fallback, allow):
    """3 when the stats all-reduce fell back to torch (on every rank) and
    --allow-stats-fallback was not given, so a multi-GPU run cannot pass
    without exercising qe_allreduce_stats; else 0."""
    if fallback and not allow:
        print(f"bench.py: the statistics all-reduce fell back to torch on every rank "
              f"({fallback}); rerun with --allow-stats-fallback to accept", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    main()
