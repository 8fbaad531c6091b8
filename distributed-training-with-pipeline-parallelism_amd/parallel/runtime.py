"""Pipeline executor: runs one rank's lowered program each ``step``.

Per action (dependency analogue: ``_PipelineScheduleRuntime._step_microbatches``,
torch schedules.py:2037-2284, and the single-stage loops schedules.py:727-994):

* ``CommGroup``  -> one grouped post (RCCL group / gloo batch).  Receives land in
  pre-allocated per-(stage, microbatch) buffers, so every receive can be posted as
  early as the global order allows and no buffer is ever re-allocated.
* ``F``          -> wait for this microbatch's receive (stream wait on GPU, not a
  host block), run the stage forward; the last stage also computes the loss
  (scaled by 1/m when ``scale_grads`` -- equivalent to the dependency's
  ``scale_grads`` div after the step, stage.py:570-584, but free).
* ``B`` / ``I`` / ``W`` -> backward (full or split).
* ``REDUCE_GRAD`` -> the stage's grad finalisation + async DP all-reduce, issued
  right after its last backward so it overlaps the rest of the flush.
* ``H``          -> (distributed head, :mod:`.headsplit`) this rank's token chunk of a
  microbatch through the LM head + loss; the last stage scatters its final-norm
  rows (``H`` messages) and its backward consumes the gathered chunk gradients
  (``D`` messages, received straight into one [T, D] buffer per microbatch).

Same-rank stage hand-offs (several virtual stages on one rank) bypass the
transport.  With ``profile=True`` every compute action is bracketed by timing
events (HIP events on GPU) and :attr:`last_timeline` / :meth:`bubble` report
the measured pipeline bubble (1 - busy / step time).
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .comm import P2P
from .debug import DepTracker, debug_level
from .headsplit import HeadPlan
from .ir import Action, CommGroup, Entry, Op, format_compute_grid
from .lower import add_head_reduce, defer_collectives, lower
from .schedules import canonical_name, generate, stage_to_rank
from .simulate import message_channel
from .stage import StageBase, specs_of
from .validate import validate

log = logging.getLogger("mipipe.pipeline")


class _Timer:
    """Per-action interval recorder: HIP events on GPU, perf_counter on CPU."""

    def __init__(self, device: torch.device):
        self.gpu = device.type == "cuda"
        self.records: List[Tuple[Action, object, object]] = []
        self.t0 = None

    def begin_step(self):
        self.records = []
        if self.gpu:
            self.t0 = torch.cuda.Event(enable_timing=True)
            self.t0.record()
        else:
            self.t0 = time.perf_counter()

    def mark(self):
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def add(self, a: Action, s, e):
        self.records.append((a, s, e))

    def finish(self) -> Tuple[List[Tuple[str, float, float]], float]:
        end = self.mark()
        if self.gpu:
            torch.cuda.synchronize()
            tl = [(str(a), self.t0.elapsed_time(s), self.t0.elapsed_time(e)) for a, s, e in self.records]
            total = self.t0.elapsed_time(end)
        else:
            tl = [(str(a), (s - self.t0) * 1e3, (e - self.t0) * 1e3) for a, s, e in self.records]
            total = (end - self.t0) * 1e3
        return tl, total


class _Range:
    """roctx range (rocprofv3 --marker-trace) + torch.profiler record_function."""

    def __init__(self, name: str):
        self.name = name
        self.rf = torch.autograd.profiler.record_function(name)

    def __enter__(self):
        self.rf.__enter__()
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(self.name)
        return self

    def __exit__(self, *exc):
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_pop()
        return self.rf.__exit__(*exc)


_LANE_STREAMS: Dict[int, List[torch.cuda.Stream]] = {}


class PipelineRuntime:
    def __init__(self, stages: Sequence[StageBase], schedule: str, n_microbatches: int, pp_rank: int,
                 pp_size: int, p2p: P2P, loss_fn: Optional[Callable] = None, scale_grads: bool = True,
                 style: str = "loop", program: Optional[Dict[int, List[Entry]]] = None, profile: bool = False,
                 orders: Optional[Dict[int, List[Action]]] = None, head: Optional[HeadPlan] = None,
                 head_costs: Optional[Dict[int, float]] = None, stage_costs: Optional[Sequence[float]] = None,
                 debug: Optional[int] = None, dp: int = 1, head_reduce_after_stage0: bool = False,
                 vote_group="pipeline"):
        self.stages: Dict[int, StageBase] = {s.stage_index: s for s in stages}
        # group over which decisions every rank must take alike are voted (the collective
        # placement): "pipeline" = the pipeline's control group; the trainer passes the
        # world's (its DP replicas run collectives with each other)
        self.vote_group = getattr(p2p, "ctrl_group", None) if vote_group == "pipeline" else vote_group
        self.schedule = canonical_name(schedule)
        self.m = n_microbatches
        self.rank = pp_rank
        self.pp = pp_size
        self.p2p = p2p
        self.loss_fn = loss_fn
        self.scale_grads = scale_grads
        self.style = style
        any_stage = stages[0]
        self.num_stages = any_stage.num_stages
        if self.num_stages % pp_size != 0:
            raise ValueError(f"{self.num_stages} stages do not divide over {pp_size} ranks")
        self.v = self.num_stages // pp_size
        if pp_size > self.num_stages:
            raise ValueError("group size must be <= number of stages (torch stage.py:173-176)")
        expected = [s for s in range(self.num_stages) if stage_to_rank(s, pp_size, style) == pp_rank]
        if sorted(self.stages) != expected:
            raise ValueError(f"rank {pp_rank} holds stages {sorted(self.stages)}, placement '{style}' expects {expected}")
        self.s2r = [stage_to_rank(s, pp_size, style) for s in range(self.num_stages)]
        self.head = head
        if program is None:
            if orders is None:
                orders = generate(self.schedule, pp_size, n_microbatches, self.v, style)
            validate(orders, pp_size, self.v, n_microbatches, style)
            self.orders = orders
            program = lower(orders, pp_size, self.v, style, head_costs=head_costs, stage_costs=stage_costs)
            if head is not None:
                program = add_head_reduce(program, after_stage0=head_reduce_after_stage0)
        else:
            self.orders = {r: [e for e in es if isinstance(e, Action) and e.op.is_compute] for r, es in program.items()}
        self.device = any_stage.device
        self.dp = int(dp)
        program = self._prove(program, p2p)
        self.program_all = program
        self.program = program[pp_rank]
        self.profile = profile
        self.timer = _Timer(self.device)
        self.last_timeline: List[Tuple[str, float, float]] = []
        self.last_step_ms: float = 0.0
        self.last_timeline_source = ""
        self._initialized = False
        self._recv_bufs: Dict[tuple, List[torch.Tensor]] = {}
        self.recv_arena_bytes = 0
        self._dh_full: Dict[int, torch.Tensor] = {}
        self._steps = 0
        self.head_losses: Dict[int, torch.Tensor] = {}
        lvl = debug_level() if debug is None else int(debug)
        self.deps: Optional[DepTracker] = DepTracker(pp_rank, lvl) if lvl > 0 else None
        # roctx / torch.profiler ranges per action ("PP:<action>", as torch schedules.py:2245)
        self.ranges = os.environ.get("MIPIPE_RANGES", "0") == "1"
        # native step replay (parallel/native_runner.py, csrc/runtime/stage_runner.cpp): once
        # every action is a captured HIP graph, one step is recorded and later steps run in C++
        self.native_enabled = os.environ.get("MIPIPE_NATIVE_RUNNER", "1") != "0"
        self.native_runner = None
        self.native_reason = "not recorded yet"
        self._tapes: Dict[bool, tuple] = {}
        self._tape_mode = False
        self._native_outputs = None
        # distributed head: ``head_reduce()`` issues the reduction of the replicated head's
        # gradient (returns work handles); the program's REDUCE_HEAD action says when
        self.head_reduce: Optional[Callable[[], list]] = None
        # microbatch lanes (set_lanes): odd microbatches on a second HIP stream
        self.lanes = 1
        self.lane_streams: List[Optional[torch.cuda.Stream]] = [None]
        self._joined = True
        self._merged: set = set()
        self._in_bufs: Dict[int, Tuple[torch.Tensor, ...]] = {}
        self._tgt_bufs: Dict[int, torch.Tensor] = {}
        self._loss_bufs: Dict[tuple, torch.Tensor] = {}
        self._install_stash_plan()

    def _install_stash_plan(self) -> None:
        """Activation-stash slots of this rank's stages under its compute order and lanes
        (parallel/stash.py): graphed stages capture each slot's microbatches into one pool,
        so a rank holds the schedule's in-flight stashes, not all m (MIPIPE_STASH_RING=0:
        one private pool per graph, the pre-round-5 behaviour)."""
        if os.environ.get("MIPIPE_STASH_RING", "1") == "0":
            return
        from .stash import plan_stash_slots
        slot, last, _ = plan_stash_slots(self.orders.get(self.rank, []), list(self.stages), self.lanes)
        for s, st in self.stages.items():
            if hasattr(st, "set_stash_plan"):
                st.set_stash_plan({mb: v for (ss, mb), v in slot.items() if ss == s},
                                  {mb: v for (ss, mb), v in last.items() if ss == s})

    # ------------------------------------------------------------------ hang-freedom
    def _prove(self, program: Dict[int, List[Entry]], p2p) -> Dict[int, List[Entry]]:
        """Choose where the step's collectives go and PROVE the resulting program cannot
        hang under the queue model that holds on this machine (simulate.check_lowered).

        Default (``MIPIPE_COLL_OVERLAP=probe``): each collective stays where it was placed
        (DP all-reduce / reduce-scatter right after the stage's last backward, head reduction
        after the rank's last head chunk) to overlap the flush.  That needs the *independent*
        queue model, so it is used only if the hardware-queue probe (parallel/queues.py)
        finds every comm stream on a queue of its own on EVERY rank (a MIN vote), with the
        native engine carrying the p2p.  Otherwise -- or with ``MIPIPE_COLL_OVERLAP=0`` --
        collectives are deferred to the end of the step (after every p2p group), and the
        program must pass the *serial* model: one FIFO per rank, the worst case of any
        stream -> hardware-queue mapping (GPU_MAX_HW_QUEUES per priority; RCCL's own
        internal streams included), so nothing about the mapping needs to be known.  With
        two p2p channels the per-direction order is proven as well (independent model), else
        the p2p falls back to one channel.  A program that no
        model admits raises instead of running."""
        from .simulate import check_lowered
        S = self.num_stages
        # receive-only posts of the native tape start at post time (ordered after the step's
        # start, not the compute stream: VERDICT r5 #6); every independent-model proof below
        # admits that (check_lowered recv_early), the serial one is unaffected by it
        # (MIPIPE_RECV_EARLY=0: ordered after the compute stream, as before)
        self.recv_early = (getattr(p2p, "kind", "") == "native" and self.device.type == "cuda"
                           and os.environ.get("MIPIPE_RECV_EARLY", "1") != "0")
        has_coll = any(isinstance(e, Action) and (e.op == Op.REDUCE_HEAD or (e.op == Op.REDUCE_GRAD and self.dp > 1))
                       for es in program.values() for e in es)
        self.coll_placement = "none"
        self.queue_report = None
        if has_coll:
            # MIPIPE_COLL_OVERLAP: probe (default) = overlap wherever the hardware-queue probe
            # clears it; 1 = same; 0 = always defer
            mode = os.environ.get("MIPIPE_COLL_OVERLAP", "probe").lower()
            kind = getattr(p2p, "kind", "")
            overlap = False
            if mode in ("1", "probe") and kind == "native" and self.device.type == "cuda":
                from .queues import comm_queues_independent
                overlap, self.queue_report = comm_queues_independent(self.device)
            elif mode in ("1", "probe") and kind in ("torch", "gloo-staged") and self._gloo(p2p):
                # gloo moves bytes on the host: a process group's collectives run on that
                # group's own worker threads, p2p on tagged unbound buffers -- no shared
                # device FIFO, i.e. the independent model (CPU plumbing, shared-GPU rehearsal)
                overlap = True
                self.queue_report = {"gloo": "host transport: independent per group"}
            if dist.is_initialized() and dist.get_world_size() > 1:
                # every rank takes the same placement: the proof below assumes
                # one program for all, so overlap only if every rank's probe cleared it
                from .comm import agree
                overlap = agree(overlap, self.vote_group, self.device)
            if overlap:
                check_lowered(program, S, channels=getattr(p2p, "channels", 1), dp=self.dp,
                              recv_early=self.recv_early)
                self.coll_placement = ("overlapped (independent queues, probed)" if kind == "native"
                                       else "overlapped (gloo host transport)")
            else:
                program = defer_collectives(program)
                self.coll_placement = "step end (serial-model proof)"
        if getattr(p2p, "channels", 1) > 1:
            try:
                check_lowered(program, S, channels=p2p.channels, dp=self.dp, recv_early=self.recv_early)
            except RuntimeError as e:
                log.warning("two-channel p2p order not provably safe (%s): single channel", e)
                p2p.use_single_channel()
        if not self.coll_placement.startswith("overlapped"):
            check_lowered(program, S, serial=True, dp=self.dp)
        return program

    @staticmethod
    def _gloo(p2p) -> bool:
        g = getattr(p2p, "group", None)
        try:
            return dist.is_initialized() and dist.get_backend(g) == "gloo"
        except Exception:   # noqa: BLE001 - no group
            return False

    # ------------------------------------------------------------------ lanes
    def set_lanes(self, n: int) -> int:
        """Run microbatch ``mb``'s compute on lane ``mb % n``: lane 0 is the compute stream,
        lane l > 0 its own HIP stream, forked from the compute stream at the start of the
        step and joined back before the gradients are reduced.  Short-token microbatches
        leave most CUs idle in every kernel (1024-token GEMMs are 96-432 tiles; 64-workgroup
        attention grids) and pay a dependent-kernel boundary per launch; two microbatches'
        graphs replayed concurrently overlap both (tools/lane_probe.py, reference model: F||F
        1.53x, B||B 1.57x, F||B 1.27x).  Each lane accumulates into its own gradient buffer
        (ParamArena.lane) -- the stage's and the distributed head's -- summed into lane 0 at
        the join; the dW side stream is turned off (a forked graph did not overlap with the
        other lane).

        Several stages per rank (interleaved): each stage's lanes are merged at its own
        REDUCE_GRAD, after which the lanes wait for the merge before running the other
        stages' remaining backwards.  PP > 1: in the 1F1B steady state F(i+w) and B(i) are both ready;
        on two lanes they overlap (a 32-sequence GPT-2 microbatch on one stream runs at 0.95x
        of two concurrent ones, profiles/r3_lane1_mbs_ab.txt).  A receive is waited for on
        the lane of the compute it feeds; a post carrying a lane's output is ordered after
        that lane (SYNC); the head's lanes are merged at REDUCE_HEAD, the stage's at
        REDUCE_GRAD.  Lane streams must have hardware queues of their own -- apart from the
        compute stream and, at PP > 1, every comm stream (the probe) -- or lanes stay off.
        Returns the lanes in use."""
        n = max(1, int(n))
        if n > 1 and (self.device.type != "cuda" or self.m < 2):
            n = 1
        self.lane_streams = [None]
        idx = (self.device.index if self.device.index is not None else torch.cuda.current_device()) if n > 1 else 0
        # one set of lane streams per device and process: HIP maps each stream onto one of
        # GPU_MAX_HW_QUEUES hardware queues when it is created, and two lanes (or a lane and
        # the compute stream) sharing a queue serialise.  torch's pool hands streams out
        # round-robin, so trainers built later in a process would get other queue mappings
        # (the reference 9-config table measured 444K tok/s for L8H8 vs 594K in a fresh
        # process); the first ones taken are reused instead
        cache = _LANE_STREAMS.setdefault(idx, [])
        main_s = torch.cuda.current_stream(idx).cuda_stream if n > 1 else None
        avoid = [main_s]
        if n > 1 and self.pp > 1:
            kind = getattr(self.p2p, "kind", "")
            if kind == "native":
                from .queues import comm_streams
                avoid += list(comm_streams(self.device).values())
            elif kind != "gloo-staged":
                n = 1       # torch p2p: its communicators' streams are not ours to probe
            # (gloo-staged -- ranks sharing one GPU in a rehearsal -- moves bytes through the
            # host on the issuing stream: no comm stream to keep clear)
        # ... and a lane must not land on the compute stream's hardware queue or another
        # lane's: the spin/flag probe (parallel/queues.py, profiles/r3_queue_probe.json)
        # found torch's second pool stream on the compute stream's queue -- the 3-lane
        # anomaly of round 2 (456K tok/s vs 495K with 2 lanes, 594K with 4).  Candidates are
        # drawn from the pool until one has a queue of its own (at most 4 per priority).
        chosen: List[torch.cuda.Stream] = []
        if n > 1:
            for c in cache:
                if len(chosen) < n - 1 and self._own_queue(c, avoid + [x.cuda_stream for x in chosen]):
                    chosen.append(c)
        tried = 0
        while n > 1 and len(chosen) < n - 1 and tried < 64:
            tried += 1
            ls = torch.cuda.Stream(device=idx)
            if ls.cuda_stream in avoid or any(ls.cuda_stream == c.cuda_stream for c in cache):
                continue
            if not self._own_queue(ls, avoid + [c.cuda_stream for c in chosen]):
                continue
            cache.append(ls)
            chosen.append(ls)
        n = min(n, len(chosen) + 1)
        if n > 1 and self.pp > 1 and self.coll_placement.startswith("overlapped"):
            # the exact program with its lane queues, under the model the placement relies on
            from .simulate import check_lowered
            check_lowered(self.program_all, self.num_stages, channels=getattr(self.p2p, "channels", 1), dp=self.dp,
                          lanes=n, recv_early=getattr(self, "recv_early", False))
        self.lanes = n
        if self.device.type == "cuda":
            # the f32 split-K planner counts 256 / n CUs per GEMM: the other lanes fill the
            # rest (+1.4 % on the reference fp32 workload with 4 lanes, r5_f32_lane_split.md)
            from ..ops.kernels import load_ext
            ext = load_ext()
            if ext is not None and hasattr(ext, "gemm_f32_set_lanes"):
                ext.gemm_f32_set_lanes(n)
        self.lane_streams += chosen[: n - 1]
        for st in self.stages.values():
            st.arena.set_lanes(n)
            if hasattr(st, "model"):
                st.model.wgrad_side = n == 1
        ha = self._head_arena()
        if ha is not None:
            ha.set_lanes(n)
        self.native_runner = None   # a recorded tape does not know about lanes
        self._tapes.clear()
        self._install_stash_plan()  # slots never shared across lanes
        return n

    def _head_arena(self):
        return getattr(self.head, "arena", None) if self.head is not None else None

    def _own_queue(self, s: torch.cuda.Stream, others) -> bool:
        """True if stream ``s`` shares a hardware queue with none of ``others`` (probe; true
        without the extension or with MIPIPE_LANE_PROBE=0)."""
        if os.environ.get("MIPIPE_LANE_PROBE", "1") == "0":
            return True
        try:
            from .queues import shares_queue
            return not any(shares_queue(int(s.cuda_stream), int(o), self.device, timeout_us=5000)[0]
                           for o in others)
        except RuntimeError:
            return True

    def _lane_ctx(self, a: Action, st):
        """Stream + gradient-lane context of one compute action (every arena it may
        accumulate into: the stage's, and the distributed head's -- which a tied
        embedding's backward on stage 0 writes too)."""
        self._cur_lane = 0
        if self.lanes == 1 or a.op not in (Op.F, Op.B, Op.I, Op.W, Op.H):
            return contextlib.nullcontext()
        ln = a.mb % self.lanes
        self._cur_lane = ln
        if ln == 0:
            return contextlib.nullcontext()
        cm = contextlib.ExitStack()
        cm.enter_context(torch.cuda.stream(self.lane_streams[ln]))
        if st is not None:
            cm.enter_context(st.arena.lane(ln))
        ha = self._head_arena()
        if ha is not None and (st is None or ha is not st.arena):
            cm.enter_context(ha.lane(ln))
        return cm

    def _order_posts_after_lanes(self, lanes_used, rec) -> None:
        """A group sending tensors produced on a lane: the compute stream (which orders the
        engine's post) first waits for that lane."""
        if self.lanes == 1:
            return
        main = torch.cuda.current_stream(self.device)
        for ln in sorted(lanes_used):
            if ln:
                ls = self.lane_streams[ln]
                main.wait_stream(ls)
                if rec is not None:
                    rec.sync(main, ls)

    def _join_head_lanes(self, rec) -> None:
        """REDUCE_HEAD: the compute stream waits for every lane, and the head arena's lane
        gradients are summed into lane 0 before its reduction is issued."""
        ha = self._head_arena()
        if self.lanes == 1 or ha is None:
            return
        main = torch.cuda.current_stream(self.device)
        for ls in self.lane_streams[1:]:
            main.wait_stream(ls)
            if rec is not None:
                rec.sync(main, ls)
        if self.head.graphs is not None and self._steps > 1:
            self.head.graphs.run(("M", 0), (), lambda ins: ha.merge_lanes())
        else:
            ha.merge_lanes()
        for ls in self.lane_streams[1:]:     # later lane work must not race the merge's zeroing
            ls.wait_stream(main)
            if rec is not None:
                rec.sync(ls, main)

    def _fork_lanes(self, rec) -> None:
        if self.lanes == 1:
            return
        main = torch.cuda.current_stream(self.device)
        for ls in self.lane_streams[1:]:
            ls.wait_stream(main)
            if rec is not None:
                rec.sync(ls, main)
        self._joined = False
        self._merged = set()

    def _join_lanes(self, rec, stage: Optional[int] = None) -> None:
        """Compute stream waits for every lane; lane gradients summed into lane 0 -- of
        ``stage`` only (its REDUCE_GRAD: with several stages per rank the others still run
        backwards on the lanes, which then wait for the merge, as it zeroes their buffers),
        or of every stage not merged yet (the end of the step).  Each stage is merged once
        per step (the fused merge also leaves its clipping sum of squares)."""
        if self.lanes == 1 or self._joined:
            return
        main = torch.cuda.current_stream(self.device)
        for ls in self.lane_streams[1:]:
            main.wait_stream(ls)
            if rec is not None:
                rec.sync(main, ls)
        todo = [stage] if stage is not None else list(self.stages)
        for s in todo:
            if s in self._merged:
                continue
            self._merged.add(s)
            st = self.stages[s]
            if getattr(st, "_graphed", lambda: False)():
                st.graphs.run(("M", 0), (), lambda ins, st=st: st.arena.merge_lanes())
            else:
                st.arena.merge_lanes()
        if len(self._merged) == len(self.stages):
            self._joined = True
        elif stage is not None:
            for ls in self.lane_streams[1:]:
                ls.wait_stream(main)
                if rec is not None:
                    rec.sync(ls, main)

    # ------------------------------------------------------------------ init
    def _needs_inference(self) -> bool:
        local = any(s.input_specs is None or s.output_specs is None for s in self.stages.values())
        if self.pp == 1 or self.p2p.group is None and not dist.is_initialized():
            return local
        flag = torch.tensor([1.0 if local else 0.0], device=self.device)
        dist.all_reduce(flag, group=self.p2p.group)
        return bool(flag.item() > 0)

    def _initialize(self, first_inputs: Optional[Tuple[torch.Tensor, ...]]):
        if self.pp > 1:
            peers = set()
            for s in self.stages:
                if s > 0:
                    peers.add(self.s2r[s - 1])
                if s < self.num_stages - 1:
                    peers.add(self.s2r[s + 1])
            if self.head is not None:  # head chunks: last-stage rank <-> every chunk rank
                last = self.s2r[self.num_stages - 1]
                if self.rank == last:
                    peers.update(self.head.ranks)
                elif self.rank in self.head.ranks:
                    peers.add(last)
            self.p2p.warmup(sorted(peers), self.rank)
        if self._needs_inference():
            prev_out = None
            for s in range(self.num_stages):
                if self.s2r[s] != self.rank:
                    continue
                st = self.stages[s]
                if s == 0:
                    if first_inputs is None:
                        raise RuntimeError("stage 0 needs inputs for shape inference")
                    args = tuple(first_inputs)
                    st.input_specs = specs_of(args)
                else:
                    if self.s2r[s - 1] == self.rank:
                        specs = prev_out
                    else:
                        specs = self.p2p.recv_specs(self.s2r[s - 1])
                    st.input_specs = specs
                    args = tuple(torch.zeros(sh, dtype=dt, device=self.device) for sh, dt in specs)
                out_specs = st.infer_output_specs(args)
                prev_out = out_specs
                if s < self.num_stages - 1 and self.s2r[s + 1] != self.rank:
                    self.p2p.send_specs(out_specs, self.s2r[s + 1])
        self._plan_recv_arena()
        self._initialized = True

    def _recv_shapes(self, key: tuple):
        """(shape, dtype) list of the tensors received under message ``key``."""
        kind = key[0]
        if kind == "H":
            h = self.head
            return [((h.chunks[key[1]], h.d_model), h.dtype)]
        _, stage, _ = key
        st = self.stages[stage]
        specs = st.input_specs if kind == "F" else st.output_specs
        return [(tuple(sh), dt) for sh, dt in specs]

    def _plan_recv_arena(self) -> None:
        """Every receive slot of the lowered program (one per (kind, stage, microbatch)
        message, plus the last stage's per-microbatch head input-gradient buffers) is
        carved out of ONE allocation made here, before the first step: the receive side
        of the 1F1B stash is sized up front from the program instead of growing lazily
        inside the step.  Slots are 256-byte aligned; ``recv_arena_bytes``
        is what it holds.  Slots stay persistent (a stage may keep its received input as
        the backward's saved activation), so graph captures and the native tape see fixed
        addresses."""
        want: List[Tuple[tuple, List]] = []
        seen = set()
        for e in self.program:
            if not isinstance(e, CommGroup):
                continue
            for op in e.ops:
                if op.action.op.is_send or op.key in seen or op.key[0] == "D":
                    continue
                seen.add(op.key)
                want.append((op.key, self._recv_shapes(op.key)))
        dh_mbs = []
        if self.head is not None and self.s2r[self.num_stages - 1] == self.rank:
            dh_mbs = list(range(self.m))
        align = 256
        off = 0
        slots = []
        for key, shapes in want:
            views = []
            for sh, dt in shapes:
                n = math.prod(sh) * torch.empty((), dtype=dt).element_size()
                views.append((off, n, sh, dt))
                off += (n + align - 1) // align * align
            slots.append((key, views))
        h = self.head
        dh_views = []
        for mb in dh_mbs:
            n = h.tokens * h.d_model * torch.empty((), dtype=h.dtype).element_size()
            dh_views.append((mb, off, n))
            off += (n + align - 1) // align * align
        self.recv_arena_bytes = off
        if off == 0:
            return
        arena = torch.empty(off, dtype=torch.uint8, device=self.device)
        self._recv_arena = arena

        def view(o, n, sh, dt):
            return arena[o:o + n].view(dt).view(sh)
        for key, views in slots:
            self._recv_bufs[key] = [view(o, n, sh, dt) for o, n, sh, dt in views]
        for mb, o, n in dh_views:
            self._dh_full[mb] = view(o, n, (h.tokens, h.d_model), h.dtype)

    def _dh_buf(self, mb: int) -> torch.Tensor:
        """[T, D] input-gradient buffer of the last stage for microbatch mb; the head
        chunks' D messages land in its row slices."""
        t = self._dh_full.get(mb)
        if t is None:
            h = self.head
            t = torch.empty(h.tokens, h.d_model, dtype=h.dtype, device=self.device)
            self._dh_full[mb] = t
        return t

    def _recv_buf(self, key: tuple) -> List[torch.Tensor]:
        kind = key[0]
        if kind == "D":
            return [self._dh_buf(key[2])[self.head.rows(key[1])]]
        buf = self._recv_bufs.get(key)
        if buf is None and kind == "H":
            h = self.head
            buf = [torch.empty(h.chunks[key[1]], h.d_model, dtype=h.dtype, device=self.device)]
            self._recv_bufs[key] = buf
        if buf is None:
            kind, stage, mb = key
            st = self.stages[stage]
            specs = st.input_specs if kind == "F" else st.output_specs
            buf = [torch.empty(sh, dtype=dt, device=self.device) for sh, dt in specs]
            self._recv_bufs[key] = buf
        return buf

    # ------------------------------------------------------------------ native replay
    def _native_possible(self, return_outputs: bool) -> bool:
        if not self.native_enabled or self.device.type != "cuda":
            return False
        if return_outputs and not all(getattr(st, "records_own_collectives", False) for st in self.stages.values()):
            return False     # autograd stages' outputs are not persistent graph buffers
        if self.deps is not None or self.ranges:
            return False
        if any(getattr(st, "graphs", None) is None for st in self.stages.values()):
            return False
        if self.head is not None and self.head.graphs is None:
            return False
        # step 1 eager, step 2 captures, step 3 (and later) replays every action
        return self._steps >= 2 and all(getattr(st, "step_id", 0) >= 2 for st in self.stages.values())

    def _loss_slot(self, key: tuple, like: torch.Tensor) -> torch.Tensor:
        buf = self._loss_bufs.get(key)
        if buf is None or buf.shape != like.shape or buf.dtype != like.dtype:
            buf = torch.empty_like(like)
            self._loss_bufs[key] = buf
        return buf

    def _persist_inputs(self, inputs, targets):
        """Copy the step's user inputs / targets into persistent per-microbatch buffers (so a
        recorded tape never points at a caller's tensor).  Runs in Python every step."""
        if inputs is not None:
            out = []
            for mb, args in enumerate(inputs):
                bufs = self._in_bufs.get(mb)
                if bufs is None or any(b.shape != a.shape for b, a in zip(bufs, args)):
                    bufs = tuple(torch.empty_like(a) for a in args)
                    self._in_bufs[mb] = bufs
                for b, a in zip(bufs, args):
                    b.copy_(a)
                out.append(bufs)
            inputs = out
        if targets is not None:
            out = []
            for mb, t in enumerate(targets):
                b = self._tgt_bufs.get(mb)
                if b is None or b.shape != t.shape:
                    b = torch.empty_like(t)
                    self._tgt_bufs[mb] = b
                b.copy_(t)
                out.append(b)
            targets = out
        return inputs, targets

    def _step_native(self, inputs, targets, losses, mode: bool = False):
        for st in self.stages.values():
            st.clear_runtime_states()
        self._steps += 1
        self._persist_inputs(inputs, targets)
        prof = self.profile
        if prof:
            self.native_runner.set_profile(True)
        try:
            self.native_runner.run()
        finally:
            if prof:
                self.native_runner.set_profile(False)
        if prof:
            # measured on the replayed tape itself: GRAPH intervals on the compute stream
            tl, total = self.native_runner.timeline()
            self.last_timeline, self.last_step_ms = [(str(a), float(s_), float(e)) for a, s_, e in tl], float(total)
            self.last_timeline_source = "native tape"
        for st in self.stages.values():
            st.post_step()
        mb_losses = {k[1]: t for k, t in self._loss_bufs.items() if k[0] == "L"}
        self.head_losses = {k[1]: t for k, t in self._loss_bufs.items() if k[0] == "H"}
        if losses is not None and mb_losses:
            losses.extend(mb_losses[i] for i in sorted(mb_losses))
        self._last_losses = mb_losses
        # the last stage's per-microbatch outputs: graph buffers the replay just rewrote
        return self._native_outputs if mode else None

    # ------------------------------------------------------------------ step
    def step(self, inputs: Optional[Sequence[Tuple[torch.Tensor, ...]]] = None,
             targets: Optional[Sequence[torch.Tensor]] = None, losses: Optional[list] = None,
             return_outputs: bool = True) -> Optional[List[Tuple[torch.Tensor, ...]]]:
        if not self._initialized:
            self._initialize(inputs[0] if inputs is not None else None)
        # one recorded tape per output mode: the compat last rank's step(return_outputs=True)
        # replays a tape whose graphs also write the logits (persistent graph outputs)
        mode = bool(return_outputs) and self.stages.get(self.num_stages - 1) is not None
        if self._tape_mode != mode:
            self._tapes[self._tape_mode] = (self.native_runner, self._native_outputs)
            self.native_runner, self._native_outputs = self._tapes.get(mode, (None, None))
            self._tape_mode = mode
        possible = self._native_possible(return_outputs)
        if possible and self.native_runner is not None:
            return self._step_native(inputs, targets, losses, mode)
        rec = None
        if possible and self.profile:
            possible = False    # the recording step itself is not the profiled path
        if possible:
            from .native_runner import TapeRecorder
            inputs, targets = self._persist_inputs(inputs, targets)
            rec = TapeRecorder(self.device)
        with (rec if rec is not None else contextlib.nullcontext()):
            out = self._step_python(inputs, targets, losses, return_outputs, rec)
        if rec is not None:
            if rec.valid:
                self.native_runner = rec.runner
                if getattr(self, "recv_early", False) and hasattr(self.native_runner, "set_recv_early"):
                    self.native_runner.set_recv_early(True)
                self._native_outputs = list(out) if (mode and out is not None) else None
                self.native_reason = f"recorded {rec.runner.size} instructions"
            elif "captured during the recording step" in rec.reason:
                # a graph this step needed for the first time (e.g. the logits-returning
                # forward of a new output mode): record again on the next step
                self.native_reason = "re-recording: " + rec.reason
            else:
                self.native_enabled = False
                self.native_reason = "disabled: " + rec.reason
                log.warning("native stage runner not used: %s", rec.reason)
        return out

    def _step_python(self, inputs, targets, losses, return_outputs, rec):
        for st in self.stages.values():
            st.clear_runtime_states()
            st.want_outputs = bool(return_outputs)
            st.n_microbatches = self.m
        recv_works: Dict[tuple, List] = {}
        send_keep: List = []
        send_tensors: Dict[tuple, Tuple[torch.Tensor, ...]] = {}
        handoff: Dict[tuple, Tuple[torch.Tensor, ...]] = {}
        outputs: Dict[int, Tuple[torch.Tensor, ...]] = {}
        mb_losses: Dict[int, torch.Tensor] = {}
        self.head_losses = {}
        head = self.head
        self._steps += 1
        reduce_works = []
        loss_scale = 1.0 / self.m if self.scale_grads else 1.0
        S = self.num_stages
        if self.profile:
            self.timer.begin_step()

        deps = self.deps

        ready = [None]   # profiling: time the last receive of the current action completed

        def wait_recv(key):
            for w in recv_works.pop(key, []):
                w.wait()
            if deps is not None:
                deps.on_wait(key)
            if self.profile:
                # busy time starts once the inputs are there (a host-blocking gloo wait on
                # CPU; on GPU an event after the stream wait)
                ready[0] = self.timer.mark()

        def read_recv(key, action):
            if deps is not None:
                deps.on_read(key, action)
            return self._recv_buf(key)

        def produce(key, tensors, action, local):
            if deps is not None:
                deps.on_produce(key, action, tensors)
            (handoff if local else send_tensors)[key] = tensors
            if not local:
                send_lane[key] = self._cur_lane

        def rng(a):
            if not self.ranges:
                return contextlib.nullcontext()
            return _Range(f"PP:{a}")

        send_lane: Dict[tuple, int] = {}
        self._cur_lane = 0
        self._fork_lanes(rec)
        for idx, e in enumerate(self.program):
            try:
                if isinstance(e, CommGroup):
                    sends, recvs, rkeys, sch, rch = [], [], [], [], []
                    self._order_posts_after_lanes({send_lane.pop(op.key, 0) for op in e.ops
                                                   if op.action.op.is_send}, rec)
                    for op in e.ops:
                        ch = message_channel(op.key)
                        if op.action.op.is_send:
                            if deps is not None:
                                deps.on_send(op.key, send_tensors)
                            ts = send_tensors.pop(op.key)
                            sends += [(t, op.peer) for t in ts]
                            sch += [ch] * len(ts)
                            send_keep.append(ts)
                        else:
                            if deps is not None:
                                deps.on_post_recv(op.key)
                            bufs = self._recv_buf(op.key)
                            recvs += [(t, op.peer) for t in bufs]
                            rch += [ch] * len(bufs)
                            rkeys += [op.key] * len(bufs)
                    sw, rw = self.p2p.post(sends, recvs, sch, rch)
                    send_keep.extend(sw)
                    for k, w in zip(rkeys, rw):
                        recv_works.setdefault(k, []).append(w)
                    continue
                a = e
                if a.op == Op.REDUCE_HEAD:
                    self._join_head_lanes(rec)
                    if self.head_reduce is not None:
                        reduce_works.extend(self.head_reduce())
                    continue
                st = self.stages.get(a.stage)
                if a.op == Op.REDUCE_GRAD:
                    if not st.has_grad_reduction(self.scale_grads):
                        # nothing to issue (no DP, scale folded into the loss): the stage's
                        # lanes are merged at the step's final join -- a join here would drain
                        # the lanes while the rank's other stages still run backwards
                        # (interleaved: one mid-step join per extra stage)
                        continue
                    self._join_lanes(rec, a.stage)
                    if rec is not None and not getattr(st, "records_own_collectives", False):
                        # an autograd stage's torch.distributed reduction: a CALL on the tape
                        from .native_runner import record_issue

                        def _rg(st=st):
                            w_ = st.reduce_grad(self.m, scaled_in_loss=self.scale_grads)
                            return [w_] if w_ is not None else []
                        reduce_works.extend(record_issue(rec, _rg))
                        continue
                    w = st.reduce_grad(self.m, scaled_in_loss=self.scale_grads)
                    if w is not None:
                        reduce_works.append(w)
                    continue
                with self._lane_ctx(a, st if a.op != Op.H else None):
                    t_s = self.timer.mark() if self.profile else None
                    ready[0] = None
                    with rng(a):
                        self._run_compute(a, st, inputs, targets, return_outputs, loss_scale, handoff, outputs,
                                          mb_losses, wait_recv, read_recv, produce)
                    if self.profile:
                        self.timer.add(a, ready[0] if ready[0] is not None else t_s, self.timer.mark())
            except Exception:
                self._report_failure(idx)
                if hasattr(self.p2p, "release_works"):
                    self.p2p.release_works()    # no handle outlives a failed step
                raise
        self._join_lanes(rec)
        if deps is not None:
            deps.finish(send_tensors, handoff)
        for w in send_keep:
            if hasattr(w, "wait"):
                w.wait()
        for w in reduce_works:
            w.wait()
        if hasattr(self.p2p, "release_works"):
            self.p2p.release_works()
        # post_step (the tied-embedding gradient sum) runs outside the recording: a replayed
        # step issues it after the tape (_step_native), so recording it would sum twice
        from .native_runner import paused
        with paused():
            for st in self.stages.values():
                st.post_step()
        if self.profile:
            self.last_timeline, self.last_step_ms = self.timer.finish()
            self.last_timeline_source = "python executor"
        if losses is not None and mb_losses:
            losses.extend(mb_losses[i] for i in sorted(mb_losses))
        self._last_losses = mb_losses
        if self.stages.get(S - 1) is not None and return_outputs:
            return [outputs[i] for i in sorted(outputs)]
        return None

    def _run_compute(self, a: Action, st, inputs, targets, return_outputs, loss_scale, handoff, outputs, mb_losses,
                     wait_recv, read_recv, produce) -> None:
        """One compute action: gather its inputs (same-rank hand-off or a waited receive),
        run it, and publish its outputs (hand-off or pending send)."""
        S = self.num_stages
        head = self.head
        if a.op == Op.F:
            key = ("F", a.stage, a.mb)
            if a.stage == 0:
                args = tuple(inputs[a.mb])
            elif key in handoff:
                args = handoff.pop(key)
            else:
                wait_recv(key)
                args = tuple(read_recv(key, a))
            tgt = targets[a.mb] if (st.is_last and targets is not None) else None
            out, loss = st.forward_mb(a.mb, args, tgt, self.loss_fn, loss_scale)
            if st.is_last and head is not None:
                # scatter the final-norm rows to the head chunks
                hn = out[0]
                for r in head.ranks:
                    produce(("H", r, a.mb), (hn[head.rows(r)],), a, r == self.rank)
            elif st.is_last:
                if return_outputs:
                    outputs[a.mb] = out
                if loss is not None:
                    if getattr(st, "_graphed", lambda: False)():
                        # graph output -> persistent loss slot (a recorded COPY on the tape)
                        from .native_runner import copy_into
                        loss = copy_into(self._loss_slot(("L", a.mb), loss), loss)
                    mb_losses[a.mb] = loss
            else:
                produce(("F", a.stage + 1, a.mb), out, a, self.s2r[a.stage + 1] == self.rank)
        elif a.op == Op.H:
            hk = ("H", a.stage, a.mb)
            if hk in handoff:
                (h_in,) = handoff.pop(hk)
            else:
                wait_recv(hk)
                (h_in,) = read_recv(hk, a)
            rows = head.rows(a.stage)
            tgt = targets[a.mb].reshape(-1)[rows]
            local_last = self.s2r[S - 1] == self.rank
            scale = loss_scale / head.tokens
            if head.graphs is not None and self._steps > 1:
                def fn(ins, local_last=local_last, mb=a.mb):
                    d = self._dh_buf(mb)[rows] if local_last else torch.empty_like(ins[0])
                    return d, head.runner(ins[0], ins[1], d, scale)
                dh, loss = head.graphs.run(("H", a.mb), (h_in, tgt), fn)
                from .native_runner import copy_into
                self.head_losses[a.mb] = copy_into(self._loss_slot(("H", a.mb), loss), loss)
            else:
                dh = self._dh_buf(a.mb)[rows] if local_last else torch.empty_like(h_in)
                self.head_losses[a.mb] = head.runner(h_in, tgt, dh, scale)
            if not local_last:
                produce(("D", a.stage, a.mb), (dh,), a, False)
        elif a.op in (Op.B, Op.I):
            key = ("B", a.stage, a.mb)
            if a.stage == S - 1 and head is not None:
                for r in head.ranks:
                    if r != self.rank:
                        wait_recv(("D", r, a.mb))
                        read_recv(("D", r, a.mb), a)
                g = (self._dh_buf(a.mb),)   # persistent per microbatch (graph-safe)
            elif a.stage == S - 1:
                g = None
            elif key in handoff:
                g = handoff.pop(key)
            else:
                wait_recv(key)
                g = tuple(read_recv(key, a))
            gin = st.backward_mb(a.mb, g) if a.op == Op.B else st.backward_input_mb(a.mb, g)
            if a.stage > 0:
                gin = tuple(x for x in gin if x is not None)
                produce(("B", a.stage - 1, a.mb), gin, a, self.s2r[a.stage - 1] == self.rank)
        elif a.op == Op.W:
            st.backward_weight_mb(a.mb)

    # ------------------------------------------------------------------ diagnostics
    def p2p_send_bytes(self) -> int:
        """Bytes this rank sends per step over the pipeline transport (activations,
        gradients, head chunks and their gradients), from the lowered program and the
        stages' static specs (valid after the first step)."""
        def nbytes(specs):
            return sum(math.prod(sh) * torch.empty((), dtype=dt).element_size() for sh, dt in specs)
        tot = 0
        for e in self.program:
            if not isinstance(e, CommGroup):
                continue
            for op in e.ops:
                if not op.action.op.is_send:
                    continue
                kind = op.key[0]
                if kind in ("H", "D"):
                    h = self.head
                    tot += h.chunks[op.key[1]] * h.d_model * torch.empty((), dtype=h.dtype).element_size()
                elif kind == "F":
                    tot += nbytes(self.stages[op.key[1] - 1].output_specs or [])
                else:
                    tot += nbytes(self.stages[op.key[1] + 1].input_specs or [])
        return int(tot)

    def busy_ms(self) -> float:
        """Busy time of the last profiled step: the union of the action intervals (with
        microbatch lanes two actions may overlap)."""
        tot, end = 0.0, float("-inf")
        for _, s_, e in sorted(self.last_timeline, key=lambda x: x[1]):
            if e <= end:
                continue
            tot += e - max(s_, end)
            end = e
        return float(tot)

    def bubble(self, step_ms: Optional[float] = None) -> float:
        """Measured bubble of the last profiled step on this rank: 1 - busy / step time
        (``step_ms``: a common step time, e.g. the max over ranks; default: this rank's)."""
        step = self.last_step_ms if step_ms is None else step_ms
        if not self.last_timeline or step <= 0:
            return float("nan")
        return max(0.0, 1.0 - self.busy_ms() / step)

    def describe(self) -> str:
        """Diagnostics for a hang report (utils/metrics.Watchdog): transport, tape state and
        the compute grid of every rank's program."""
        grid = {r: [e for e in es if isinstance(e, Action)] for r, es in self.program_all.items()}
        head = (f"pipeline rank {self.rank}/{self.pp}: schedule {self.schedule}, m={self.m}, v={self.v}, "
                f"p2p={getattr(self.p2p, 'kind', '?')}, native runner: {self.native_reason}, steps run: {self._steps}")
        return head + "\n" + format_compute_grid(grid)

    def _report_failure(self, idx: int) -> None:
        grid = {r: [e for e in es if isinstance(e, Action)] for r, es in self.program_all.items()}
        step = sum(1 for e in self.program[:idx] if isinstance(e, Action))
        log.error("pipeline rank %d failed at action #%d (%s)\n%s", self.rank, idx, self.program[idx],
                  format_compute_grid(grid, error_step=step, error_rank=self.rank))
