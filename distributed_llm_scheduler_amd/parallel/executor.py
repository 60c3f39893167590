"""Per-rank DAG executor.

One process per GPU (``torch.distributed`` world, backend ``nccl`` = RCCL on ROCm, or
``gloo`` for the CPU fake-device backend). Each rank executes its :class:`Program`:

* activations live in ONE preallocated slab per rank at statically planned offsets
  (program.py); parameters in a second slab whose size is the per-GPU memory cap;
* ``load`` copies a parameter group host(pinned)->HBM unless the arena region still holds it
  from the previous step (steady-state residency). On GPU the copy runs on a side copy
  stream, issued as soon as the last kernel that used an overlapping arena region has been
  enqueued (hipEvent fork), and the compute stream waits for it only at the load's own
  position — parameter refills overlap the kernels in between (``DLS_PREFETCH=1``; default
  in order on the compute stream). A refill is ONE DMA of the group's pinned host image;
* ``recv``/``send`` are RCCL point-to-point ops (parallel/comm.py): the sends and receives a
  rank posts at one program point go out as ONE group (``batch_isend_irecv``, one
  ncclGroupStart/End); RCCL runs them on its own stream ordered after the producing kernels,
  and the consumer waits stream-side (``work.wait()``), so transfers overlap the next
  independent kernels; a sent buffer is only overwritten (by a kernel or by a recv from
  another peer) after its send completes (waits planned statically, ``Instr.wait_sends``).
  The same primitives also run over the single-GPU loopback hub (several ranks in one
  process, parallel/loopback.py), which checks that stream ordering on one device;
* ``run`` launches the (fused) kernel group through :mod:`ops` — HIP kernels on GPU;
* programs without p2p ops are captured once into a hipGraph (``torch.cuda.CUDAGraph``)
  and replayed, removing per-kernel host launch cost from the step.

``profile=True`` records a start/stop hipEvent pair per kernel group, giving a measured
per-GPU Gantt (same layout as the reference's simulated one, visu.py:206-248).
"""
from __future__ import annotations

import math
import os
import time
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from ..core.task import Task
from ..ops import tuning as _tuning
from ..models.params import ParamStore, group_layout
from ..utils.tracing import Roctx
from . import lifetime
from .comm import make_comm
from .program import Program


@dataclass
class StepStats:
    wall_ms: float = 0.0
    kernels: int = 0
    sends: int = 0
    recvs: int = 0
    bytes_sent: int = 0
    bytes_recv: int = 0
    param_fills: int = 0
    bytes_filled: int = 0
    peer_fills: int = 0   # parameter groups received from a peer's HBM over xGMI
    bytes_peer: int = 0
    timeline: List[Tuple[str, float, float]] = field(default_factory=list)  # (group, start_ms, end_ms)
    events: List[Tuple[str, str, float, float]] = field(default_factory=list)  # (name, category, start, end)


class _REvent:
    """An event of the native step runner (index into its own hipEvents), used in place of a
    torch Event while a step is recorded."""
    __slots__ = ("idx",)

    def __init__(self, idx: int):
        self.idx = idx


class _RWork:
    """A p2p op of the native step runner: ``wait()`` records the wait."""
    __slots__ = ("runner", "idx")

    def __init__(self, runner, idx: int):
        self.runner, self.idx = runner, idx

    def wait(self):
        self.runner.add_work_wait(self.idx)


class _Recorder:
    """Records one steady-state step's device actions into a native ``StepRunner`` (csrc/kernels/
    runner.cpp) instead of executing them (a dry run of the Python issue loop)."""

    def __init__(self, runner):
        self.r = runner
        self.n_events = 0
        self.carry: Dict[int, int] = {}  # load index -> event index of its cross-step fill

    def event(self, carry_load: Optional[int] = None) -> _REvent:
        if carry_load is not None:
            if carry_load not in self.carry:
                self.carry[carry_load] = self.n_events
                self.n_events += 1
            return _REvent(self.carry[carry_load])
        self.n_events += 1
        return _REvent(self.n_events - 1)


# native step runner for segment-replayed programs: "auto" (default) keeps it unless a
# comm-free program's steps measure faster from the Python issue loop (Llama-3-8B at a 13.8 GB
# cap: 55.3 vs 52.1 ms; at 15.5 GB the runner wins, 17.1 vs 18.0 — profiles/r3_final), "1"
# always, "0" never
RUNNER_MODE = os.environ.get("DLS_RUNNER", "auto")
RUNNER = RUNNER_MODE != "0"
# CPU backend (tests): the runner replays the recorded step with kernel groups as Python
# callbacks and p2p through the gloo ProcessGroup — the same action list as on the GPU
RUNNER_CPU = os.environ.get("DLS_RUNNER_CPU", "0") == "1"


def synthetic_tokens(name: str, n: int, vocab: int, seed: int = 1234) -> torch.Tensor:
    """Deterministic synthetic token ids for external input ``name`` — identical on every
    rank and in tests, whichever rank happens to own the consuming task."""
    g = torch.Generator().manual_seed((zlib.crc32(name.encode()) ^ seed) & 0x7FFFFFFF)
    return torch.randint(0, vocab, (n,), generator=g, dtype=torch.int32)


# device p2p transport: expert-parallel edges move only the routed rows (DAGExecutor._plan_routed_edges)
EP_ROUTED = os.environ.get("DLS_EP_ROUTED", "1") == "1"
FOLD_MAX_K = 1024  # fold a preceding norm into the GEMM only up to this K (see DAGExecutor._gemm)
# widest norm input whose statistics a producer GEMM hands over (beyond it: a norm kernel)
HANDOFF_MAX_K = int(os.environ.get("DLS_HANDOFF_MAX_K", str(FOLD_MAX_K)))
GUARD_BYTES, GUARD_VALUE = 4096, 0xA5  # debug-mode canary after each arena slab
# producer GEMMs emit row statistics for the next folded norm (GPU); DLS_STATS_HANDOFF=0 disables
STATS_HANDOFF = os.environ.get("DLS_STATS_HANDOFF", "1") != "0"
# the embedding kernel hands layer 0's folded norm its rows' statistics too (0: that norm's GEMM
# accumulates them in its main loop)
EMBED_STATS = os.environ.get("DLS_EMBED_STATS", "1") != "0"
# parameter refills on a side copy stream, hoisted to the earliest safe point (GPU), and the
# step then runs eagerly (the branches of a captured hipGraph execute one after the other on
# this stack, benchmarks/bench_graph_concurrency.py). "auto" (default): for planned-residency
# programs whose streamed loads are issued ahead (Program.prefetch); "1": every program with
# loads — measured slower for replayed policy traces (gpt2-medium, 8 GB reference-cost cap,
# MRU_spec: 20.4 vs 19.4 ms: their evictions free a region just before it is re-filled);
# "0": never (the plans then issue no loads ahead either, runtime.plan)
PREFETCH = os.environ.get("DLS_PREFETCH", "auto")
# one grouped launch pair per MoE layer for the experts co-located on this rank (GPU)
MOE_BATCH = os.environ.get("DLS_MOE_BATCH", "1") != "0"
# one grouped launch pair per co-run span (program.plan_coruns): a layer's experts on this rank
# over every request (expert parallelism with data-parallel attention)
MOE_XBATCH = os.environ.get("DLS_MOE_XBATCH", "1") != "0"
# MoE routing in one launch (router + align, ops.moe_route) and the grouped gate/up GEMM
# gathering its token rows itself (no permute kernel); 0 restores the separate launches
MOE_FUSED_ROUTE = os.environ.get("DLS_MOE_FUSED_ROUTE", "1") != "0"
# an unfolded norm (K > FOLD_MAX_K) computed by the block that produces its input: the split-K
# reduce of the residual GEMM (or the MoE combine) owns whole rows and writes norm(row) too
POST_NORM = os.environ.get("DLS_POST_NORM", "1")  # "0" off, "1" every producer, "gemm" residual GEMMs only
# parameter refills: "pull" = the host-pull kernel reads the pinned group image over the host
# link (benchmarks/bench_h2d.py: 50-56 GB/s from 2.4 MB up, 32 GB/s at 0.25 MB, on 32-64
# workgroups), "dma" = hipMemcpyAsync (42-51 GB/s, 15 GB/s at 0.25 MB)
REFILL = os.environ.get("DLS_REFILL", "pull")
# a group the policy evicted counts as gone (default: the executed refill traffic is exactly
# the policy's decisions); DLS_VICTIM_REUSE=1 instead re-uses its bytes when the region was not
# overwritten before the group is loaded again at the same offset
VICTIM_REUSE = os.environ.get("DLS_VICTIM_REUSE", "0") == "1"
REFILL_BLOCKS = int(os.environ.get("DLS_REFILL_BLOCKS", "64"))
# a pre-norm MLP block (folded norm + fc1 + GELU, then fc2 + residual) as ONE launch
# (ops.mlp_fused, csrc/kernels/gemm_fused.hip) where the shape fits its grid (GPU)
MLP_FUSED = os.environ.get("DLS_MLP_FUSED", "0") == "1"
# a pre-norm attention block (folded norm + QKV GEMM, causal MHA, out-proj + residual) as ONE
# launch (ops.attn_block, csrc/kernels/attn_block.hip) where the shape fits (GPU). Off by default:
# measured 36.3 vs 25.3 us for the three launches at GPT-2's block (profiles/r6_status/
# attn_block_stamps_v3.txt: the heaviest query tiles wait for the last q/k/v tile of every row)
ATTN_BLOCK = os.environ.get("DLS_ATTN_BLOCK", "0") == "1"
# device p2p transport: every P2P_CHECK_EVERY-th step the rank's error word is mirrored into
# pinned host memory (an asynchronous copy, no host sync) and the mirror of the previous check
# is read; a set word fails the step loudly (TransportError). check_transport() reads it
# synchronously (the CLI, the bench and the evaluation harness call it after their steps).
P2P_CHECK_EVERY = max(1, int(os.environ.get("DLS_P2P_CHECK_EVERY", "8")))


class TransportError(RuntimeError):
    """A device-transport wait gave up after DLS_P2P_TIMEOUT_S (devp2p.py): the wait stopped
    spinning and the step went on, so this rank's outputs of that step are wrong."""


class DAGExecutor:
    def __init__(self, tasks: Sequence[Task], program: Program, store: ParamStore, device: torch.device,
                 model_cfg=None, use_graph: bool = True, pg=None, seed: int = 1234, autotune: bool = True,
                 trace: bool = False, debug: bool = False, model_name: Optional[str] = None,
                 input_parts: Optional[Dict[str, List[str]]] = None,
                 requests: Optional[Dict[str, Tuple[str, int, int]]] = None):
        self.tasks = {t.id: t for t in tasks}
        # the model whose per-model GEMM choices (ops/gemm_tuning.json model_overrides) this
        # executor's launches use: set around each of its steps, captures and refinements, so
        # executors of different models in one process do not change each other's choices
        self.model_name = model_name if model_name is not None else getattr(model_cfg, "name", None)
        self.prog = program
        self.store = store
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.cfg = model_cfg
        self.pg = pg
        self.comm = make_comm(pg)  # p2p transport: torch.distributed (RCCL / gloo) or the loopback hub
        # whole-step hipGraph for comm-free programs without copy-stream refills; the others
        # replay hipGraph SEGMENTS (runs of kernel groups) between their eager RCCL / copy steps
        self.use_graph = use_graph and self.gpu
        self.seed = seed
        # merged micro-batches (runtime.plan merge_mb): an external input made of several
        # requests' token ids, and request prefix -> (merged prefix, batch rows) for output()
        self.input_parts = dict(input_parts or {})
        self.requests = dict(requests or {})
        self.trace = trace  # roctx range per instruction (eager steps; a graph replay is one range)
        self.debug = debug  # canary guards after every arena + non-finite check of outputs, per step
        self._local_consumed = None
        self.dtype = torch.bfloat16
        self._graph = None
        self._views: Dict[str, torch.Tensor] = {}     # activation views (output task -> tensor)
        self._params: Dict[str, Dict[str, torch.Tensor]] = {}  # pid -> {tensor name -> view}
        self._wflat: Dict[str, torch.Tensor] = {}               # tensor name -> resident view
        self._derived_cache: Dict[tuple, tuple] = {}             # (weight, ptr) -> (colsum, bias') for folded norms
        # weights read by more than one KIND of op (GPT-2's tied wte: embedding gather + LM head)
        # are never transformed in place: their folded form lives in a private buffer. Tasks of
        # one kind reading one weight (request replicas, sequence chunks) apply the same
        # transform and share it in place.
        self._side: Dict[str, torch.Tensor] = {}                 # weight -> private derived copy
        kinds: Dict[str, set] = {}
        for t in tasks:
            if t.op is not None:
                for v in set(x for x in t.op.weights.values() if isinstance(x, str)):
                    kinds.setdefault(v, set()).add(t.op.kind)
        self._w_users: Dict[str, int] = {v: len(k) for v, k in kinds.items()}
        # GPU, host-image refills: a transformed weight's bytes are written back into a private
        # copy of its group's pinned image, so every later refill restores the TRANSFORMED
        # weight and its (colsum, bias') stay valid wherever the group lands (no re-derivation
        # kernels per refill)
        self._img_override: Dict[str, torch.Tensor] = {}         # pid -> pinned image
        self._derived_named: Dict[str, tuple] = {}                # weight -> (colsum, bias')
        self._tensor_home: Dict[str, Tuple[str, int]] = {}        # weight -> (pid, byte offset in group)
        self._refills_memo: Optional[bool] = None
        self._valid: List[Tuple[int, int, str]] = []  # param arena regions holding data
        # group -> (offset, bytes) its views in _params / _wflat point at; a fill that overwrites
        # any part of that region unmaps the group (its views would read another group's bytes)
        self._region: Dict[str, Tuple[int, int]] = {}
        self._inputs: Dict[str, torch.Tensor] = {}
        self._scratch_bufs: Dict[str, torch.Tensor] = {}
        self._moe_memo: Dict[tuple, object] = {}
        self._stats_out: Dict[str, torch.Tensor] = {}   # producer output -> fp32 [M, 2] row stats it emits
        self._ext_stats: Dict[str, torch.Tensor] = {}   # the same buffers, by the tensor a norm reads
        self._stats_slab: Optional[torch.Tensor] = None
        self._moe_ptrs: Dict[tuple, torch.Tensor] = {}
        self._pending_sends: Dict[int, object] = {}  # send instruction index -> RCCL work
        self._param_recv: Dict[str, object] = {}     # group -> RCCL work of its peer fill
        self._started = False
        self._steps_done = 0
        self.launches: Optional[int] = None  # kernel launches of one captured step (hipGraph kernel nodes)
        self._rope: Dict[Tuple[int, int, float], Tuple[torch.Tensor, torch.Tensor]] = {}
        self.last = StepStats()
        self._err_mirror: Optional[torch.Tensor] = None  # device transport: pinned copy of the error word
        self._attn_sync: Optional[torch.Tensor] = None   # one-launch attention blocks' counters + error word
        self._attn_mirror: Optional[torch.Tensor] = None
        self._watch_n = 0
        self._setup()
        self._exp_ids: Dict[str, torch.Tensor] = {}
        self._routed_in: Dict[str, torch.Tensor] = {}  # received hidden state -> local experts (int32)
        self._routed_out: set = set()                   # received expert outputs (compact rows)
        self._deferred: Dict[str, object] = {}          # their receives, pulled by the MoE code
        self._pull_at: Dict[int, List[str]] = {}        # instruction -> hidden states pulled after it
        if self._device_p2p:
            self.comm.attach(self)  # peers pull from this rank's arenas (IPC exchange across processes)
            if EP_ROUTED:
                self._plan_routed_edges()
        self._plan_ep_capacity()
        if autotune and self.gpu:
            _tuning.set_model(self.model_name)
            _tuning.ensure_tuned(self.gemm_shapes(), self.device)

    # ------------------------------------------------------------------ setup
    def _setup(self) -> None:
        p = self.prog
        dev = self.device
        g = GUARD_BYTES if self.debug else 0
        self._act_full = torch.empty(max(p.act_arena_bytes, 256) + g, dtype=torch.uint8, device=dev)
        self._param_full = torch.empty(max(p.param_arena_bytes, 256) + g, dtype=torch.uint8, device=dev)
        self.act_slab = self._act_full[:self._act_full.numel() - g]
        self.param_slab = self._param_full[:self._param_full.numel() - g]
        if g:
            self._act_full[-g:].fill_(GUARD_VALUE)
            self._param_full[-g:].fill_(GUARD_VALUE)
        for tid, off in p.act_offset.items():
            t = self.tasks[tid]
            shape = tuple(t.op.out_shape) if t.op is not None and t.op.out_shape else (p.act_bytes[tid] // 2,)
            pad = t.op.attrs.get("ld_pad", 1) if t.op is not None else 1
            cols = (shape[-1] + pad - 1) // pad * pad
            rows = math.prod(shape[:-1])
            v = self.act_slab[off:off + 2 * rows * cols].view(self.dtype).view(rows, cols)
            if cols != shape[-1]:
                v = v[:, :shape[-1]]  # padded row stride (16-B aligned rows for vector stores)
            self._views[tid] = v.view(shape)
        # workspace for intra-group temporaries (attention qkv / o, mlp gate_up ...)
        ws = 0
        for ins in p.instrs:
            if ins.op == "run":
                ws = max(ws, self._workspace_bytes(ins))
        self._ws_full = torch.empty(max(ws, 256) + g, dtype=torch.uint8, device=dev)
        self.ws_slab = self._ws_full[:self._ws_full.numel() - g]
        if g:
            self._ws_full[-g:].fill_(GUARD_VALUE)
        # external inputs (token ids per request replica)
        for ins in p.instrs:
            if ins.op != "run":
                continue
            for tid in ins.group:
                op = self.tasks[tid].op
                for name in op.inputs:
                    if name not in self.tasks and name not in self._inputs:
                        # a sequence chunk's embedding reads its slice of the whole request
                        M = op.attrs.get("tokens_total", math.prod(op.out_shape[:-1]))
                        vocab = self.cfg.vocab_size if self.cfg is not None else 50257
                        parts = self.input_parts.get(name)
                        if parts:  # merged micro-batches: the requests' own token ids, in row order
                            self._inputs[name] = torch.cat([synthetic_tokens(q, M // len(parts), vocab, self.seed)
                                                            for q in parts]).to(dev)
                        else:
                            self._inputs[name] = synthetic_tokens(name, M, vocab, self.seed).to(dev)
        if self.gpu and STATS_HANDOFF:
            self._plan_stats_handoff()
        self._zero_in_embedding = False
        self._zero_run = None  # the run whose embedding launch zeroes the statistics slab
        if self._stats_slab is not None:
            runs = [i for i in p.instrs if i.op == "run"]
            first = self.tasks[runs[0].group[0]] if runs else None
            self._zero_in_embedding = first is not None and first.op.kind == "embedding"
            self._zero_run = runs[0] if self._zero_in_embedding else None
        self._plan_moe_batches()
        self._plan_moe_xbatch()
        self._hoist: Dict[int, List[int]] = {}
        self._await: Dict[str, object] = {}  # group -> copy-stream event its first reader waits on
        self._segments: Dict[int, Tuple[int, object]] = {}  # segment start -> (end, hipGraph)
        self._capture_plan: Optional[Dict[int, int]] = None  # set while capture_segments runs
        self._seg_pool = None
        self._cap_stream = None  # side stream segment captures run on (_capture_segment)
        self._rec: Optional[_Recorder] = None   # set while a step is recorded for the runner
        self._runner = None                     # native StepRunner replaying the recorded step
        self.issue_mode: Optional[str] = None  # "runner" / "python" for segment-replayed programs
        self._graph_exec: Optional[int] = None  # the whole-step hipGraphExec (graph_launch)
        self._fast = None  # (launch, exec, device, stats) of a captured whole step
        self._runner_stats: Optional[StepStats] = None
        self._stream_kind = 0                   # 0 compute / 1 copy stream (recording of fills)
        self._carry_at: Dict[int, List[int]] = {}  # instr -> next step's loads issued after it
        self._carry: Dict[int, object] = {}  # next step's loads already issued -> their events
        self._copy_stream = None
        # (device p2p transport: refills stay in order on the compute stream, so the whole step —
        # refills, kernels and edges — is ONE hipGraph)
        if self.gpu and (PREFETCH == "1" or (PREFETCH == "auto" and p.prefetch)) \
                and any(i.op == "load" for i in p.instrs) and not self._device_p2p:
            self._plan_prefetch()
            self._copy_stream = torch.cuda.Stream(self.device)
        self._post_norm: Dict[int, Task] = {}  # producer run -> the next norm it also writes
        self._norm_given: Dict[int, str] = {}  # consumer run -> its norm task, already written
        self._pn: Optional[Task] = None        # set by _issue_run for the run in flight
        self._pn_given: Optional[str] = None   # its consumer: the norm its producer wrote (if it did)
        self._pn_done: Optional[str] = None    # the norm the last producer actually wrote
        if POST_NORM not in ("0", False) and self._copy_stream is None:
            self._plan_post_norm()  # (pairs are adjacent runs: no p2p between producer and consumer)
        self._plan_mlp_fused()

    def _plan_post_norm(self) -> None:
        """Pair each norm that the next group would run as its own pass (its width is above
        FOLD_MAX_K on GPU, so it is not folded into the consumer GEMM) with the group that
        produces its input right before it: a residual block (attention / SwiGLU MLP, whose
        split-K residual GEMM reduces whole rows) or the MoE combine (a workgroup per row).
        That producer writes the normalised rows too — into the norm's own output when the
        norm is a group of its own (Mixtral's post-attention norm feeds the router and the
        experts), else into the consumer's norm scratch buffer. Only runs with nothing but
        parameter loads / evictions between them (no kernel can touch the scratch rows); the
        producer writes the norm only while the norm's weights are resident (every steady-state
        step; a first step that loads them later lets the consumer run the norm itself)."""
        ins = self.prog.instrs
        norms = ("layernorm", "rmsnorm")
        runs = [i for i, x in enumerate(ins) if x.op == "run"]
        for i, j in zip(runs, runs[1:]):
            P, Q = ins[i], ins[j]
            if any(ins[k].op not in ("load", "evict") for k in range(i + 1, j)):
                continue
            pg = [self.tasks[t] for t in P.group]
            qg = [self.tasks[t] for t in Q.group]
            N = qg[0]
            if N.op is None or N.op.kind not in norms or not N.op.inputs or N.op.inputs[0] != pg[-1].id:
                continue
            width = N.op.out_shape[-1]
            if self.gpu and (width <= FOLD_MAX_K or width > 8192 or N.op.inputs[0] in self._ext_stats):
                continue  # folded into the consumer GEMM, or wider than a reduce row holds
            head = pg[1] if (pg[0].op.kind in norms and len(pg) > 1) else pg[0]
            block = len(pg) > 1 and pg[-1].op.kind == "residual" and head.op.kind in ("attention", "swiglu_mlp")
            combine = len(pg) == 1 and head.op.kind == "moe_combine" and POST_NORM != "gemm"
            if not (block or combine) or (len(qg) == 1 and N.id not in self._views):
                continue
            self._post_norm[i] = N
            self._norm_given[j] = N.id

    def _post_norm_out(self, out2d: torch.Tensor):
        """(y, w, b, kind, eps) for ops' ``post_norm`` when the run in flight feeds a norm
        (``out2d``: the producer's output rows, which the post-norm reads whole)."""
        N = self._pn
        if N is None or not out2d.is_contiguous():
            return None
        W = N.op.weights
        if not all(self._resident(q) for q in N.params_needed):
            # the norm's weight group is not mapped with valid bytes right now (it is loaded
            # after this run, e.g. the first step or a cold-lowered capped program): the
            # consumer runs the norm itself
            return None
        y = self._flat(self._views[N.id]) if N.id in self._views else self._scratch("norm", out2d.shape)
        self._pn_done = N.id
        return (y, self._w(W["w"]), self._w(W["b"]) if "b" in W else None, N.op.kind, N.op.attrs.get("eps", 1e-5))

    def _plan_moe_batches(self) -> None:
        """Every expert node of one MoE layer that sits on this rank, back to back in the
        program (only parameter loads between them), runs as ONE grouped launch pair (gate/up
        with SwiGLU, then down) instead of two GEMMs per expert: grid = experts x column
        tiles, so the layer's whole expert weight stream is one chip-wide launch. GPU only,
        all experts of the layer here, and a program without evictions or peer parameter
        loads (parameters never move, so the span's loads can be applied at the batch's first
        node); activation p2p elsewhere in the program does not matter."""
        self._moe_batch: Dict[int, Tuple[List[int], List[int]]] = {}
        self._moe_skip: set = set()
        self._moe_batched_ids: set = set()
        self._moe_bufs: Dict[int, tuple] = {}
        self._gate_route: Dict[str, Tuple[int, int]] = {}  # router task -> (E, top-k): GEMM + routing fused
        ins = self.prog.instrs
        if not self.gpu or not MOE_BATCH or any(i.op == "evict" or (i.op == "load" and i.peer >= 0) for i in ins):
            return  # (p2p elsewhere in the program is fine: parameters never move)

        def expert_of(j):
            x = ins[j]
            if x.op != "run" or len(x.group) != 1:
                return None
            t = self.tasks[x.group[0]]
            return t if t.op is not None and t.op.kind == "moe_expert" else None

        i = 0
        while i < len(ins):
            t0 = expert_of(i)
            if t0 is None:
                i += 1
                continue
            key = tuple(t0.op.inputs[:2])
            members, loads, j = [i], [], i + 1
            while j < len(ins):
                t = expert_of(j)
                if ins[j].op == "load":
                    loads.append(j)
                elif t is not None and tuple(t.op.inputs[:2]) == key:
                    members.append(j)
                else:
                    break
                j += 1
            E = t0.op.attrs["n_experts"]
            experts = sorted(self.tasks[ins[m].group[0]].op.attrs["expert"] for m in members)
            if len(members) > 1 and experts == list(range(E)):
                self._moe_batch[i] = (members, [ld for ld in loads if ld < members[-1]])
                self._moe_skip |= set(members[1:])
                self._moe_batched_ids |= {ins[m].group[0] for m in members}
                if MOE_FUSED_ROUTE:  # the layer's router node computes its logits AND the routing
                    self._gate_route[t0.op.inputs[1]] = (E, t0.op.attrs["top_k"])
            i = j

    def _plan_moe_xbatch(self) -> None:
        """The program's co-run spans (program.plan_coruns) issued as ONE grouped launch pair
        at the span's first run: one MoE layer's expert nodes placed on this rank, over every
        request. With data-parallel attention and expert parallelism every request's routed
        rows reach this GPU in the same layer, so each expert's weights stream once per layer
        instead of once per request. Re-checked against the instructions: only sends,
        parameter loads and receives no member reads lie between the members."""
        self._xbatch: Dict[int, Tuple[List[int], List[int]]] = {}
        self._xskip: set = set()
        self._xfirst: Dict[str, List[int]] = {}  # first member's output task -> member indices
        self._xbatched_ids: set = set()
        self._xbufs: Dict[int, tuple] = {}
        self._xblock: Dict[str, Tuple[int, int, int]] = {}  # hidden state -> (block, rows, width)
        self._xpb_shape: Tuple[int, int] = (0, 1)  # the batches' token matrix (one, shared)
        if not MOE_XBATCH:
            return
        ins = self.prog.instrs
        run_at = {x.task: i for i, x in enumerate(ins) if x.op == "run"}
        for span in self.prog.coruns:
            idx = [run_at.get(t) for t in span]
            if None in idx or any(k in self._moe_batch or k in self._moe_skip for k in idx):
                continue
            ts = [self.tasks[ins[k].group[0]] for k in idx]
            if len({t.op.inputs[1] for t in ts}) > ops.XBATCH_MAX_REQ or len(ts) > ops.XBATCH_MAX_GROUPS:
                continue
            reads = {d for t in ts for d in t.dependencies}
            between = [k for k in range(idx[0], idx[-1]) if k not in idx]
            if any(not (ins[k].op in ("send", "load") or (ins[k].op == "recv" and ins[k].task not in reads))
                   or (ins[k].op == "load" and ins[k].peer >= 0) for k in between):
                continue
            self._xbatch[idx[0]] = (idx, [k for k in between if ins[k].op == "load"])
            reqs = list(dict.fromkeys(t.op.inputs[0] for t in ts))
            R = math.prod(self.tasks[reqs[0]].op.out_shape[:-1]) * ts[0].op.attrs["top_k"]
            H = self.tasks[reqs[0]].op.out_shape[-1]
            for q, h in enumerate(reqs):  # (a routed hidden state is pulled straight into its block)
                self._xblock[h] = (q, R, H)
            if len(reqs) * R * H > math.prod(self._xpb_shape):
                self._xpb_shape = (len(reqs) * R, H)
            self._xskip |= set(idx[1:])
            self._xfirst[ins[idx[0]].task] = idx
            self._xbatched_ids |= {t.id for t in ts}

    def _run_moe_xbatch(self, i: int, stats: StepStats) -> None:
        """A co-run span as one grouped launch pair: group g = (request q, expert e) with the
        device-side row range of q's routing; each request's expert-sorted rows are gathered (over
        the device transport: pulled, the local experts' routed rows only) into its block of one
        token matrix, and one index launch maps the groups' rows into it (no host sync). The
        groups of one expert share its weights: the launches run each weight panel's groups side
        by side on one XCD with the weights cached, so a panel streams from HBM once per layer
        whatever the request count."""
        members, loads = self._xbatch[i]
        for ld in loads:  # fixed regions (no evictions): map the span's groups up front
            self._load(ld, self.prog.instrs[ld].param, stats)
        tasks = [self.tasks[self.prog.instrs[m].group[0]] for m in members]
        # blocks in program order, as _plan_moe_xbatch numbered them (_xblock: eager pulls)
        reqs = list(dict.fromkeys((t.op.inputs[0], t.op.inputs[1]) for t in tasks))
        tasks.sort(key=lambda t: t.op.attrs["expert"])  # an expert's groups side by side
        a = tasks[0].op.attrs
        E, K, F = a["n_experts"], a["top_k"], a["ffn"]
        routes = [self._moe_route(r, E, K) for _, r in reqs]
        R = routes[0][2].numel()
        xp = self._scratch("moe_xpb", self._xpb_shape)
        for q, (h, r) in enumerate(reqs):
            self._moe_permuted(h, r, E, K, out=xp[q * R:(q + 1) * R])
        bufs = self._xbufs.get(i)
        if bufs is None:  # (first, eager step: never allocated during capture)
            bufs = (torch.zeros(len(tasks) + 1, dtype=torch.int32, device=self.device),
                    torch.zeros(len(reqs) * R, dtype=torch.int32, device=self.device))
            self._xbufs[i] = bufs
        offsets, a_rows = bufs
        ops.moe_xbatch_index([rt[4] for rt in routes], [reqs.index((t.op.inputs[0], t.op.inputs[1])) for t in tasks],
                             [t.op.attrs["expert"] for t in tasks], [q * R for q in range(len(reqs))], offsets, a_rows)
        w13 = [self._prep(t.op.weights["w_gate_up"], None, None, interleave=True)[0] for t in tasks]
        w2 = [self._w(t.op.weights["w_down"]) for t in tasks]
        outs = [self._flat(self._views[t.id]) for t in tasks]
        hbuf = self._scratch("moe_h", (len(reqs) * R, F))
        hint = max(1, R // E)
        if not self.gpu:
            ops.gemm_grouped(xp, w13, offsets, act="swiglu", out=hbuf, rows_hint=hint, a_rows=a_rows)
            ops.gemm_grouped(hbuf, w2, offsets, outs=outs, rows_hint=hint)
            return
        ptrs = tuple(w.data_ptr() for w in w13 + w2 + outs)
        cached = self._moe_bufs.get(("x", i))
        if cached is None or cached[0] != ptrs:
            mk = lambda ts: torch.tensor([x.data_ptr() for x in ts], dtype=torch.int64, device=self.device)  # noqa: E731
            cached = (ptrs, mk(w13), mk(w2), mk(outs))
            self._moe_bufs[("x", i)] = cached
        ops.gemm_grouped(xp, w13, offsets, act="swiglu", out=hbuf, w_ptrs=cached[1], rows_hint=hint, a_rows=a_rows,
                         shared_weights=True)
        ops.gemm_grouped(hbuf, w2, offsets, outs=outs, w_ptrs=cached[2], out_ptrs=cached[3], rows_hint=hint,
                         shared_weights=True)

    def _plan_mlp_fused(self) -> None:
        """Pairs (fc1 group i, fc2 group j) of a pre-norm MLP block that run as ONE launch:
        ``norm+linear+gelu`` followed by ``linear+residual`` reading its output, the norm's row
        statistics handed over by its input's producer, only parameter loads between the two
        (applied at i: a program without evictions or peer loads, whose regions never move)."""
        self._mlp_fused: Dict[int, int] = {}
        self._mlp_skip: set = set()
        self._mlp_loads: Dict[int, List[int]] = {}
        self._mlp_sync = None
        ins = self.prog.instrs
        if not (self.gpu and MLP_FUSED) or any(x.op == "evict" or (x.op == "load" and x.peer >= 0) for x in ins):
            return
        for i in range(len(ins) - 1):
            a = ins[i]
            if a.op != "run" or a.kind != "layernorm+linear+gelu":
                continue
            j = i + 1
            while j < len(ins) and ins[j].op == "load":
                j += 1
            if j >= len(ins):
                continue
            b = ins[j]
            if b.op != "run" or b.kind != "linear+residual":
                continue
            g1, g2 = [self.tasks[t] for t in a.group], [self.tasks[t] for t in b.group]
            if g2[0].dependencies != [a.task] or b.wait_sends or j in self._post_norm \
                    or self._ext_stats.get(g1[0].op.inputs[0]) is None:
                continue
            x_shape, h_shape = g1[0].op.out_shape, g1[-1].op.out_shape
            M = math.prod(x_shape[:-1])
            if not ops.mlp_fused_ok(M, x_shape[-1], h_shape[-1], g2[-1].op.out_shape[-1]):
                continue
            self._mlp_fused[i] = j
            self._mlp_skip.add(j)
            self._mlp_loads[i] = list(range(i + 1, j))
            if self._mlp_sync is None or self._mlp_sync.numel() < 2 * M // 64 + 1:
                self._mlp_sync = torch.zeros(2 * M // 64 + 1, dtype=torch.int32, device=self.device)

    def _run_mlp_fused(self, i: int) -> None:
        for ld in self._mlp_loads[i]:  # fixed regions (no evictions): fc2's groups mapped up front
            self._load(ld, self.prog.instrs[ld].param, StepStats())
        a, b = self.prog.instrs[i], self.prog.instrs[self._mlp_fused[i]]
        norm, fc1 = self.tasks[a.group[0]], self.tasks[a.group[1]]
        fc2, tail = self.tasks[b.group[0]], self.tasks[b.group[-1]]
        src = norm.op.inputs[0]
        W1, cs, b1 = self._prep(fc1.op.weights["w"], norm, fc1.op.weights.get("b"))
        W2 = self._w(fc2.op.weights["w"])
        b2 = self._w(fc2.op.weights["b"]) if "b" in fc2.op.weights else None
        res = self._flat(self._x([d for d in tail.op.inputs if d != fc2.id][0]))
        ops.mlp_fused(self._flat(self._x(src)), W1, b1, cs, self._ext_stats[src], norm.op.kind,
                      norm.op.attrs.get("eps", 1e-5), self._flat(self._views[a.task]), W2, b2, res,
                      self._flat(self._views[tail.id]), self._stats_out.get(tail.id), self._mlp_sync)

    def _run_moe_batch(self, i: int, stats: StepStats) -> None:
        members, loads = self._moe_batch[i]
        for ld in loads:  # fixed regions (no evictions): map the span's groups up front
            self._load(ld, self.prog.instrs[ld].param, stats)
        tasks = sorted((self.tasks[self.prog.instrs[m].group[0]] for m in members), key=lambda t: t.op.attrs["expert"])
        a = tasks[0].op.attrs
        E, K = a["n_experts"], a["top_k"]
        route = self._moe_route(tasks[0].op.inputs[1], E, K)
        off, src = route[4], route[2]
        if MOE_FUSED_ROUTE:  # tokens: the gate/up GEMM gathers its rows by src
            x, rows = self._flat(self._x(tasks[0].op.inputs[0])), src
        else:
            x, rows = self._moe_permuted(tasks[0].op.inputs[0], tasks[0].op.inputs[1], E, K), None
        R, F = src.numel(), a["ffn"]
        w13 = [self._prep(t.op.weights["w_gate_up"], None, None, interleave=True)[0] for t in tasks]
        w2 = [self._w(t.op.weights["w_down"]) for t in tasks]
        outs = [self._flat(self._views[t.id]) for t in tasks]
        ptrs = tuple(w.data_ptr() for w in w13 + w2 + outs)
        cached = self._moe_bufs.get(i)
        if cached is None or cached[0] != ptrs:
            mk = lambda ts: torch.tensor([x.data_ptr() for x in ts], dtype=torch.int64, device=self.device)  # noqa: E731
            cached = (ptrs, mk(w13), mk(w2), mk(outs))
            self._moe_bufs[i] = cached
        hbuf = self._scratch("moe_h", (R, F))
        ops.gemm_grouped(x, w13, off, act="swiglu", out=hbuf, w_ptrs=cached[1], rows_hint=max(1, R // E), a_rows=rows)
        ops.gemm_grouped(hbuf, w2, off, outs=outs, w_ptrs=cached[2], out_ptrs=cached[3], rows_hint=max(1, R // E))

    def _plan_prefetch(self) -> None:
        """For every ``load`` at instruction i: the earliest point it may start — right after
        the last earlier instruction that touches an overlapping arena region (a kernel
        group using a parameter group resident there, or an earlier load into it). The
        copy is issued there on the copy stream; the mapping switch stays at i.

        Loads whose region is free from the step start (hoisted to -1) are carried over the
        step boundary: the previous step issues them right after the LAST instruction that
        touches their region (``_carry_at``), so the next step's first refills run under the
        current step's tail kernels instead of stalling the next step's first kernel."""
        # groups resident from a warm start occupy their regions until evicted
        region: Dict[str, Tuple[int, int]] = {pid: (off, group_layout(self.store.groups[pid])[0])
                                              for pid, off in self.prog.start_resident.items()}
        touches: List[Tuple[int, List[Tuple[int, int]]]] = []
        for i, ins in enumerate(self.prog.instrs):
            if ins.op == "load" and ins.peer >= 0:  # fetched from a peer in the message order, never hoisted
                off = self.prog.param_offset.get((i, ins.param))
                if off is not None:
                    size = group_layout(self.store.groups[ins.param])[0]
                    region[ins.param] = (off, size)
                    touches.append((i, [(off, size)]))
                continue
            if ins.op == "psend":  # reads the group's region
                touches.append((i, [(ins.param_off, group_layout(self.store.groups[ins.param])[0])]))
                continue
            if ins.op == "load":
                off = self.prog.param_offset.get((i, ins.param))
                if off is None:
                    continue
                size = group_layout(self.store.groups[ins.param])[0]
                j = -1
                for ti, regs in reversed(touches):
                    if any(o < off + size and off < o + n for o, n in regs):
                        j = ti
                        break
                self._hoist.setdefault(j, []).append(i)
                region[ins.param] = (off, size)
                touches.append((i, [(off, size)]))
            elif ins.op == "run":
                used = set()
                for tid in ins.group:
                    used |= self.tasks[tid].params_needed
                regs = [region[q] for q in used if q in region]
                if regs:
                    touches.append((i, regs))
        for i in self._hoist.get(-1, []):  # cross-step: after the region's last toucher
            off = self.prog.param_offset[(i, self.prog.instrs[i].param)]
            size = group_layout(self.store.groups[self.prog.instrs[i].param])[0]
            last = max(ti for ti, regs in touches if any(o < off + size and off < o + n for o, n in regs))
            self._carry_at.setdefault(last, []).append(i)

    def _plan_stats_handoff(self) -> None:
        """Pair every folded norm with the GEMM that produces its input on this rank: the
        producer's epilogue emits each output row's (sum, sum of squares) into a small fp32
        buffer (zeroed once per step), and the consumer GEMM reads them instead of
        re-deriving them in its main loop — the norm then costs nothing at any K."""
        producers = {ins.task: ins for ins in self.prog.instrs if ins.op == "run"}

        def emits(ins) -> bool:
            grp = [self.tasks[t] for t in ins.group]
            lead_norm = grp[0].op.kind in ("layernorm", "rmsnorm") and len(grp) > 1
            head = grp[1] if lead_norm else grp[0]
            if head.op.kind in ("attention", "attn_sp", "swiglu_mlp"):
                return True
            if head.op.kind == "embedding" and len(grp) == 1:
                return EMBED_STATS  # the embedding kernel writes its rows' statistics (a wave per row)
            # a plain GEMM group writes its output with an un-folded, non-SwiGLU GEMM
            return head.op.kind == "linear" and not lead_norm and head.op.attrs.get("act") != "swiglu"

        need = []
        for ins in self.prog.instrs:
            if ins.op != "run":
                continue
            grp = [self.tasks[t] for t in ins.group]
            if len(grp) > 1 and grp[0].op.kind in ("layernorm", "rmsnorm"):
                src = grp[0].op.inputs[0]
                pi = producers.get(src)
                # measured (MI355X, scripts/gpu_ab.sh): a win where the norm would otherwise be
                # folded with main-loop statistics (K <= FOLD_MAX_K: GPT-2 0.857 -> 0.832 ms);
                # at K = 4096 the separate norm kernel is cheaper than the split-K reduce
                # epilogue work (Llama-3-8B 9.89 vs 9.96 ms)
                width = self.tasks[src].op.out_shape[-1] if src in self.tasks else 0
                if pi is not None and emits(pi) and src not in need and width <= HANDOFF_MAX_K:
                    need.append(src)
        if not need:
            return
        # an embedding's statistics lead the slab: the embedding kernel zeroes the rest of it
        # in the same launch (regions written there must not be zeroed there)
        need.sort(key=lambda t: 0 if self.tasks[t].op.kind == "embedding" else 1)
        rows = {t: math.prod(self.tasks[t].op.out_shape[:-1]) for t in need}
        self._stats_slab = torch.zeros(sum(2 * r for r in rows.values()), dtype=torch.float32, device=self.device)
        off = 0
        for t in need:
            buf = self._stats_slab[off:off + 2 * rows[t]]
            self._stats_out[t] = buf
            self._ext_stats[t] = buf
            off += 2 * rows[t]

    def gemm_shapes(self):
        """(M, N, K) of every GEMM this rank's program launches (for autotuning)."""
        shapes = set()
        for ins in self.prog.instrs:
            if ins.op != "run":
                continue
            for t in (self.tasks[x] for x in ins.group):
                shapes |= self._gemm_shapes_of(t)
        return sorted(shapes)

    def _gemm_shapes_of(self, t):
        """(M, N, K, variant) of the GEMMs task ``t`` launches (see ops.tuning.tag)."""
        shapes = set()
        op = t.op
        if op is not None and op.out_shape:
            M = math.prod(op.out_shape[:-1])
            g = self.store.groups
            spec = {s.name: s for pid in t.params_needed for s in g[pid].tensors}
            names = [(k, v) for k, v in op.weights.items() if k.startswith("w") and isinstance(v, str)]
            for wk, n in names:
                if n in spec and len(spec[n].shape) == 2 and op.kind not in ("embedding", "layernorm", "rmsnorm"):
                    N, K = spec[n].shape
                    if op.kind == "moe_expert":
                        hint = max(1, M * op.attrs["top_k"] // op.attrs["n_experts"])
                        grouped = t.id in self._moe_batched_ids or t.id in self._xbatched_ids
                        v = "g" if grouped else "r"  # grouped launch or one range
                        shapes.add((hint, N, K, ("s" if wk == "w_gate_up" else "") + v))
                    elif op.kind == "swiglu_mlp" and wk == "w_gate_up":
                        shapes.add((M, N, K, "s"))
                    else:
                        shapes.add((M, N, K, ""))
        return shapes

    def _workspace_bytes(self, ins) -> int:
        grp = [self.tasks[x] for x in ins.group]
        t = grp[1] if len(grp) > 1 and grp[0].op is not None and grp[0].op.kind in ("layernorm", "rmsnorm") \
            else grp[0]
        if t.op is None:
            return 0
        k = t.op.kind
        M = math.prod(t.op.out_shape[:-1]) if t.op.out_shape else 0
        a = t.op.attrs
        if k == "attention":
            D = a["head_dim"]
            qkv = M * (a["n_head"] + 2 * a["n_kv_head"]) * D
            return 2 * (qkv + M * a["n_head"] * D) + 512
        if k == "swiglu_mlp":
            F = a["ffn"]
            return 2 * (M * 2 * F + M * F) + 512
        if k == "attn_sp":
            # gathered K/V of the visible chunks + the attention output
            D = a["head_dim"]
            keys = M * len(t.op.inputs)
            return 2 * (keys * 2 * a["n_kv_head"] * D + M * a["n_head"] * D) + 1024
        if k == "moe":
            return 0
        return 0

    def _ws(self, offset_elems: int, shape) -> torch.Tensor:
        n = math.prod(shape)
        base = (offset_elems * 2 + 255) // 256 * 256
        return self.ws_slab[base:base + 2 * n].view(self.dtype).view(shape)

    # ------------------------------------------------------------- parameters
    def _group_views(self, instr_index: int, pid: str):
        off = self.prog.param_offset.get((instr_index, pid))
        if off is None:
            raise RuntimeError(f"parameter group {pid} did not fit the per-GPU parameter budget")
        return self._views_at(off, pid)

    def _views_at(self, off: int, pid: str):
        total, layout = group_layout(self.store.groups[pid])
        views = {}
        for spec, sub in layout:
            n = spec.numel
            views[spec.name] = self.param_slab[off + sub:off + sub + 2 * n].view(self.dtype).view(spec.shape)
        return off, total, layout, views

    def _map(self, pid: str, off: int, total: int, views) -> None:
        """Point the group's tensor names at its views in the arena region [off, off+total)."""
        self._params[pid] = views
        self._wflat.update(views)
        self._region[pid] = (off, total)

    def _unmap(self, pid: str) -> None:
        for name in self._params.pop(pid, {}):
            self._wflat.pop(name, None)
        self._region.pop(pid, None)

    def _overwrite(self, off: int, total: int, pid: str) -> None:
        """Region [off, off+total) is about to receive group ``pid``: every OTHER group mapped
        over any part of it loses its mapping and its validity (a later reader must load it
        again; a stale view would silently read ``pid``'s bytes)."""
        self._valid = [r for r in self._valid if r[0] + r[1] <= off or off + total <= r[0]]
        for q, (o, n) in list(self._region.items()):
            if q != pid and o < off + total and off < o + n:
                self._unmap(q)

    def _resident(self, pid: str) -> bool:
        """Is group ``pid`` mapped AND do its arena bytes currently hold it? (Not while a peer
        fill of it is still in flight: its bytes are being written by the receive.)"""
        r = self._region.get(pid)
        return r is not None and (r[0], r[1], pid) in self._valid and pid not in self._param_recv

    # --- device actions: executed, or recorded for the native step runner (self._rec) ---
    def _new_event(self, timing: bool = False, carry_load: Optional[int] = None):
        if self._rec is not None:
            return self._rec.event(carry_load)
        return torch.cuda.Event(enable_timing=timing)

    def _record(self, ev, stream=None) -> None:
        if self._rec is not None:
            self._rec.r.add_event_record(ev.idx, 1 if stream is not None and stream is self._copy_stream else 0)
        elif stream is not None:
            ev.record(stream)
        else:
            ev.record()

    def _stream_wait(self, stream, ev) -> None:
        if self._rec is not None:
            self._rec.r.add_event_wait(ev.idx, 1 if stream is self._copy_stream else 0)
        else:
            stream.wait_event(ev)

    @property
    def _device_p2p(self) -> bool:
        """Edges moved by kernels (parallel/devp2p.py): the whole step is one hipGraph."""
        return self.comm is not None and self.comm.kind == "device"

    def _isend(self, buf, peer, key=None):
        if self._rec is not None:
            return _RWork(self._rec.r, self._rec.r.add_send(buf, peer))
        if self._device_p2p:
            return self.comm.isend(buf, peer, key)
        return self.comm.isend(buf, peer)

    def _irecv(self, buf, peer, key=None):
        if self._rec is not None:
            return _RWork(self._rec.r, self._rec.r.add_recv(buf, peer))
        if self._device_p2p:
            return self.comm.irecv(buf, peer, key)
        return self.comm.irecv(buf, peer)

    def _p2p_group(self, ops_):
        """Post [(is_send, buffer, peer, key)] as ONE group (one ncclGroupStart/End); a work per
        op. ``key`` names the message for the device transport (devp2p.edge_slots)."""
        if self._rec is not None:
            r = self._rec.r
            if len(ops_) > 1:
                r.add_group_begin()
            ws = [_RWork(r, r.add_send(b, p) if snd else r.add_recv(b, p)) for snd, b, p, _ in ops_]
            if len(ops_) > 1:
                r.add_group_end()
            return ws
        if self._device_p2p:
            return self.comm.batch(ops_)
        return self.comm.batch([(snd, b, p) for snd, b, p, _ in ops_])

    def _act_region(self, tid: str) -> torch.Tensor:
        """The bytes of task ``tid``'s activation region, as the program sized it."""
        off = self.prog.act_offset[tid]
        return self.act_slab[off:off + self.prog.act_bytes[tid]]

    def _fill(self, off, total, layout, views, pid, stats: StepStats, dma: bool = False) -> bool:
        """Copy the group into its arena region unless the region already holds it. ``dma``:
        through the copy engines even when refills are pulled by a kernel (a copy overlapping
        kernels must not hold CUs: a pull kernel's workgroups delay every co-running GEMM
        until the copy ends — Llama-3-8B FFN 0.20 -> 0.60 ms beside a 16-block pull)."""
        if (off, total, pid) in self._valid:
            return False  # region still holds this group (steady-state residency)
        self._overwrite(off, total, pid)
        for spec, _ in layout:  # these weights are original again: drop stale folded-norm state
            if spec.name not in self._derived_named:
                self._derived_cache.pop((spec.name, views[spec.name].data_ptr()), None)
                self._derived_cache.pop(("side", spec.name, views[spec.name].data_ptr()), None)
        img = self._img_override.get(pid)
        if img is None and self.gpu:
            img = self.store.group_image(pid)
        rec = self._rec
        if img is not None and self.gpu and REFILL == "pull" and not dma and img.is_pinned():
            if rec is not None:
                rec.r.add_pull(self.param_slab[off:off + total], img, total, REFILL_BLOCKS, self._stream_kind)
            else:
                ops.ext().host_pull(self.param_slab[off:off + total], img, REFILL_BLOCKS)
        elif img is not None:  # one DMA of the whole group image
            if rec is not None and not self.gpu:  # CPU runner: a callback copy
                dst = self.param_slab[off:off + total]
                rec.r.add_pycall(lambda: dst.copy_(img))
            elif rec is not None:
                rec.r.add_memcpy(self.param_slab[off:off + total], img, total, self._stream_kind)
            else:
                self.param_slab[off:off + total].copy_(img, non_blocking=True)
        else:
            if rec is not None and not self.gpu:  # CPU runner: a callback fill
                rec.r.add_pycall(lambda: [self.store.fill(sp.name, views[sp.name]) for sp, _ in layout])
                self._valid.append((off, total, pid))
                stats.param_fills += 1
                stats.bytes_filled += total
                return True
            if rec is not None:
                raise RuntimeError("step runner: a parameter refill without a host image cannot be recorded")
            for spec, _ in layout:
                self.store.fill(spec.name, views[spec.name])
        self._valid.append((off, total, pid))
        stats.param_fills += 1
        stats.bytes_filled += total
        return True

    def _prefetch(self, i: int, after, stats: StepStats, pending: Dict[int, object], events,
                  carry: bool = False) -> None:
        """Issue load i's copy on the copy stream behind the compute-stream event ``after``
        (``carry``: for the next step's start, issued under this step's tail)."""
        pid = self.prog.instrs[i].param
        off, total, layout, views = self._group_views(i, pid)
        if (off, total, pid) in self._valid:
            pending[i] = None
            return
        cs = self._copy_stream
        self._stream_wait(cs, after)
        with torch.cuda.stream(cs):
            t0 = self._mark() if events is not None else None
            self._stream_kind = 1
            try:
                self._fill(off, total, layout, views, pid, stats, dma=True)
            finally:
                self._stream_kind = 0
            done = self._new_event(events is not None, carry_load=i if carry else None)
            self._record(done, cs)
        if events is not None:
            events.append((pid, "load", t0, done))
        pending[i] = done

    def _await_fill(self, pid: str) -> None:
        """The compute stream waits for ``pid``'s copy-stream fill (issued ahead by _prefetch)."""
        done = self._await.pop(pid, None)
        if done is not None:
            self._stream_wait(torch.cuda.current_stream(self.device), done)

    def _load(self, instr_index: int, pid: str, stats: StepStats) -> None:
        off, total, layout, views = self._group_views(instr_index, pid)
        if (off, total, pid) in self._valid:
            self._map(pid, off, total, views)
            return  # region still holds this group (steady-state residency)
        self._fill(off, total, layout, views, pid, stats)
        self._map(pid, off, total, views)

    def _evict(self, pid: str) -> None:
        """The policy dropped the group: its bytes count as gone (a later load re-fills it even
        if the region was not reused meanwhile), so the executed refill traffic is exactly the
        policy's evict/reload decisions."""
        self._unmap(pid)
        if not VICTIM_REUSE:
            self._valid = [r for r in self._valid if r[2] != pid]

    def _w(self, name: str) -> torch.Tensor:
        t = self._wflat.get(name)
        if t is None:
            raise KeyError(f"parameter tensor {name} is not resident on rank {self.prog.rank}")
        return t

    # ---------------------------------------------------------------- kernels
    def _x(self, name: str) -> torch.Tensor:
        v = self._views.get(name)
        if v is not None:
            return v
        return self._inputs[name]

    def _flat(self, t: torch.Tensor) -> torch.Tensor:
        return t.reshape(-1, t.shape[-1])

    def _rope_tables(self, S: int, D: int, theta: float):
        key = (S, D, theta)
        if key not in self._rope:
            self._rope[key] = ops.rope_tables(S, D, theta, self.device)
        return self._rope[key]

    # --- derived weights, recomputed after every real fill of W (cache keyed by W's address) ---
    def _prep(self, w_name: str, norm: Optional[Task] = None, b_name: Optional[str] = None,
              interleave: bool = False, rope_perm: Optional[tuple] = None):
        """(W, colsum, bias) for the GEMM on weight ``w_name``, transformed IN PLACE once per
        fill: a preceding norm folded in (W' = W*gain, colsum(W'), bias' = bias + W.beta) and/or
        the gate/up rows interleaved for the SwiGLU epilogue (every per-row vector with them),
        and/or the q/k rows of each head pair-interleaved for the RoPE epilogue
        (``rope_perm = (n_q_heads, n_k_heads, head_dim)``). W is read by this fused group only,
        so overwriting it is safe."""
        W = self._w(w_name)
        if self._w_users.get(w_name, 1) > 1 and (norm is not None or interleave or rope_perm is not None):
            return self._prep_side(W, w_name, norm, b_name, interleave, rope_perm)
        named = self._derived_named.get(w_name)
        if named is not None:  # the arena holds the transformed weight (refilled from its image)
            return W, named[0], named[1]
        key = (w_name, W.data_ptr())
        d = self._derived_cache.get(key)
        if d is None:
            bias = self._w(b_name) if b_name else None
            cs = None
            if norm is not None:
                nw = self._w(norm.op.weights["w"])
                nb = self._w(norm.op.weights["b"]) if "b" in norm.op.weights else None
                wd, cs, bd = ops.derive_norm_gemm(W, nw, nb, bias)
                bias = bd if (bias is not None or nb is not None) else None
            else:
                wd = W
            if interleave:
                wd = ops.interleave_gate_up(wd)
                cs = ops.interleave_gate_up(cs) if cs is not None else None
                bias = ops.interleave_gate_up(bias) if bias is not None else None
            if rope_perm is not None:
                perm = ops.rope_pair_perm(*rope_perm, wd.shape[0]).to(wd.device)
                wd = wd[perm].contiguous()
                cs = cs[perm].contiguous() if cs is not None else None
                bias = bias[perm].contiguous() if bias is not None else None
            if wd is not W:
                W.copy_(wd)
            d = (cs, bias)
            self._derived_cache[key] = d
            if wd is not W:
                self._persist_transform(w_name, W, d)
        return W, d[0], d[1]

    def _prep_side(self, W, w_name, norm, b_name, interleave, rope_perm):
        """_prep for a weight other tasks also read: the transformed weight is written to a
        private HBM buffer (derived again whenever the source group is re-filled)."""
        key = ("side", w_name, W.data_ptr())
        d = self._derived_cache.get(key)
        if d is None:
            bias = self._w(b_name) if b_name else None
            cs = None
            wd = W
            if norm is not None:
                nw = self._w(norm.op.weights["w"])
                nb = self._w(norm.op.weights["b"]) if "b" in norm.op.weights else None
                wd, cs, bd = ops.derive_norm_gemm(W, nw, nb, bias)
                bias = bd if (bias is not None or nb is not None) else None
            if interleave:
                wd = ops.interleave_gate_up(wd)
                cs = ops.interleave_gate_up(cs) if cs is not None else None
                bias = ops.interleave_gate_up(bias) if bias is not None else None
            if rope_perm is not None:
                perm = ops.rope_pair_perm(*rope_perm, wd.shape[0]).to(wd.device)
                wd = wd[perm].contiguous()
                cs = cs[perm].contiguous() if cs is not None else None
                bias = bias[perm].contiguous() if bias is not None else None
            buf = self._side.get(w_name)
            if buf is None or buf.shape != W.shape:
                buf = torch.empty_like(W)
                self._side[w_name] = buf
            buf.copy_(wd)
            d = (cs, bias, buf)
            self._derived_cache[key] = d
        return d[2], d[0], d[1]

    def _refills(self) -> bool:
        """Does this rank's program re-fill any parameter group after its first step (steady-state
        host refills, or groups received from a peer)?"""
        if self._refills_memo is None:
            from .program import steady_fill_bytes
            pb = {pid: group_layout(g)[0] for pid, g in self.store.groups.items()}
            self._refills_memo = (steady_fill_bytes(self.prog, pb) > 0
                                  or any(i.op == "load" and i.peer >= 0 for i in self.prog.instrs))
        return self._refills_memo

    def _persist_transform(self, w_name: str, W: torch.Tensor, d: tuple) -> None:
        """Write the transformed weight into a private copy of its group's host image (pinned
        on GPU; once, in an eager step). Every later refill — from the host image, or from a
        peer that holds the group in the same form — then carries the transformed bytes."""
        if self.gpu and torch.cuda.is_current_stream_capturing():
            return
        if not self._refills():
            return  # nothing is ever re-filled: a private (pinned) host image would be dead weight
        if not self._tensor_home:
            for gid, grp in self.store.groups.items():
                for spec, sub in group_layout(grp)[1]:
                    self._tensor_home[spec.name] = (gid, sub)
        pid, sub = self._tensor_home[w_name]
        img = self._img_override.get(pid)
        if img is None:
            base = self.store.group_image(pid)
            if base is None or (self.gpu and not base.is_pinned()):
                return  # device-initialised store: nothing is ever re-filled from the host
            img = base.clone().pin_memory() if self.gpu else base.clone()
            self._img_override[pid] = img
        nb = W.numel() * W.element_size()
        img[sub:sub + nb].copy_(W.reshape(-1).view(torch.uint8))  # blocking D2H
        self._derived_named[w_name] = d

    def _gemm(self, x, w_name, b_name, norm: Optional[Task], act=None, residual=None, out=None, rope=None,
              rope_perm=None, stats_out=None):
        """One GEMM node, optionally with a preceding norm folded in (GPU, K <= FOLD_MAX_K:
        the in-kernel row statistics cost more than a separate norm pass at larger K and
        force split-K off; measured on MI355X, Llama-3-8B K=4096: 109 vs 45+8 us).
        ``act="swiglu"``: W is a [gate; up] weight, interleaved on first use. ``rope`` /
        ``rope_perm``: RoPE in the epilogue over pair-interleaved q/k rows."""
        sw = act == "swiglu"
        ext = self._ext_stats.get(norm.op.inputs[0]) if norm is not None else None
        shared = self._w_users.get(w_name, 1) > 1
        if norm is not None and self.gpu and (ext is not None or x.shape[-1] <= FOLD_MAX_K) \
                and not (shared and self._refills()):
            # (a shared weight's folded copy is private: a step that re-fills its group would
            # need the derivation inside the replayed step, so such programs run the norm)
            # folded norm: statistics handed over by x's producer (any K, split-K allowed), or
            # accumulated in this GEMM's main loop (K <= FOLD_MAX_K)
            W, cs, bd = self._prep(w_name, norm, b_name, interleave=sw, rope_perm=rope_perm)
            return ops.linear_norm(x, W, cs, bd, norm.op.kind, norm.op.attrs.get("eps", 1e-5), act=act,
                                   residual=residual, out=out, rope=rope, ext_stats=ext)
        if norm is not None and self._pn_given == norm.id:  # x's producer wrote the normalised rows
            x = self._scratch("norm", x.shape)
            norm = None
        if norm is not None:
            nw = self._w(norm.op.weights["w"])
            xn = self._scratch("norm", x.shape)
            if norm.op.kind == "layernorm":
                ops.layernorm(x, nw, self._w(norm.op.weights["b"]), norm.op.attrs.get("eps", 1e-5), out=xn)
            else:
                ops.rmsnorm(x, nw, norm.op.attrs.get("eps", 1e-5), out=xn)
            x = xn
        if sw or rope_perm is not None:
            W, _, bias = self._prep(w_name, None, b_name, interleave=sw, rope_perm=rope_perm)
        else:
            W, bias = self._w(w_name), (self._w(b_name) if b_name else None)
            if w_name in self._derived_named or (w_name, W.data_ptr()) in self._derived_cache:
                # another reader folded a norm into / reordered this weight IN PLACE (_prep): the
                # plain GEMM would compute with W' silently (the fold decision must be
                # the same for every reader of a shared weight, e.g. DLS_HANDOFF_MAX_K > FOLD_MAX_K
                # with a replica whose input came from a peer without row statistics)
                raise RuntimeError(f"{w_name}: unfolded GEMM over a weight another reader transformed in place")
        return ops.linear(x, W, bias, act=act, residual=residual, out=out, rope=rope, stats_out=stats_out)

    def _scratch(self, tag: str, shape) -> torch.Tensor:
        """Reusable per-rank buffer (allocated on first use, i.e. in an eager warm-up step,
        never during hipGraph capture)."""
        n = math.prod(shape)
        buf = self._scratch_bufs.get(tag)
        if buf is None or buf.numel() < n:
            buf = torch.empty(n, dtype=self.dtype, device=self.device)
            self._scratch_bufs[tag] = buf
        return buf[:n].view(shape)

    def _moe_route(self, r_name: str, E: int, top_k: int):
        """Routing of one MoE layer on this rank from its router logits, computed ONCE per step
        and shared by every expert (and the combine) placed here: top-k experts and gates,
        the expert-sorted order (src rows, slot of each (token, k), per-expert offsets)."""
        key = ("route", r_name)
        r = self._moe_memo.get(key)
        if r is None:
            logits = self._flat(self._x(r_name))
            if MOE_FUSED_ROUTE:
                r = ops.moe_route(logits, top_k, E)  # one launch on GPU
            else:
                idx, gate = ops.moe_router(logits, top_k)
                r = (idx, gate) + tuple(ops.moe_align(idx, E))
            self._moe_memo[key] = r
        return r

    def _moe_permuted(self, h_name: str, r_name: str, E: int, top_k: int, out: Optional[torch.Tensor] = None):
        """The layer's hidden state in expert-sorted row order (once per step and request; into
        ``out`` when given: a cross-request batch's block)."""
        key = ("perm", h_name, r_name)
        xp = self._moe_memo.get(key)
        if xp is None:
            route = self._moe_route(r_name, E, top_k)
            src = route[2]
            rw = self._deferred.pop(h_name, None)
            cap = self._ep_unpack.get(h_name)
            if cap is not None and (h_name, cap[0]) in self._ep_full:
                cap = None
            if cap is not None:  # capacity edge: the routed rows arrived packed — unpack them
                H = self.tasks[h_name].op.out_shape[-1]
                xp = out if out is not None else self._scratch("moe_xp/" + h_name.split("/")[0], (src.numel(), H))
                peer, experts, rows, erows = cap
                f = self._ep_groups[(h_name, peer)]
                ops.moe_pack(xp, src, route[4], [(self._flat(self._x(h_name))[:rows], rows, experts, f,
                                                  [erows] * len(experts), [f] * len(experts))], self._ep_ovf,
                             unpack=True)
            elif rw is not None:  # device transport: pull the local experts' routed rows only
                H = self.tasks[h_name].op.out_shape[-1]
                # one buffer per request: another request's experts may run between two of this one's
                xp = out if out is not None else self._scratch("moe_xp/" + h_name.split("/")[0], (src.numel(), H))
                rw.pull_rows(xp.view(-1).view(torch.uint8), H * xp.element_size(), src.to(torch.int32), route[4],
                             self._routed_in[h_name], src.numel())
            else:
                xp = ops.moe_permute(self._flat(self._x(h_name)), src, out=out)
            self._moe_memo[key] = xp
        elif out is not None and xp.data_ptr() != out.data_ptr():
            out.copy_(xp)
            xp = out
        return xp

    def _moe_expert(self, t: Task, out: torch.Tensor) -> None:
        """One expert node: its routed rows (a device-side range of the expert-sorted rows) run
        the gate_up GEMM with the SwiGLU epilogue and the down GEMM, which writes them
        COMPACTLY to rows 0..count-1 of this node's [M, H] output (the layer's combine node
        gathers them by slot; no per-expert zero-filled [M, H] pass)."""
        a, W = t.op.attrs, t.op.weights
        E, K, e = a["n_experts"], a["top_k"], a["expert"]
        off = self._moe_route(t.op.inputs[1], E, K)[4]
        xp = self._moe_permuted(t.op.inputs[0], t.op.inputs[1], E, K)
        rows = off[e:e + 2]
        R, F = xp.shape[0], a["ffn"]
        hint = max(1, R // E)
        hbuf = self._scratch("moe_h", (R, F))
        W13, _, _ = self._prep(W["w_gate_up"], None, None, interleave=True)
        ops.linear(xp, W13, act="swiglu", out=hbuf, rows=rows, rows_hint=hint)
        ops.linear(hbuf, self._w(W["w_down"]), out=out, rows=rows, rows_hint=hint, compact=True)

    def _moe_combine(self, t: Task, out: torch.Tensor) -> None:
        """residual + gate-weighted gather of the compact expert outputs (inputs: expert
        nodes..., router, residual)."""
        a = t.op.attrs
        ins_ = t.op.inputs
        experts, r_name, res_name = ins_[:-2], ins_[-2], ins_[-1]
        idx, gate, _, slot, off = self._moe_route(r_name, a["n_experts"], a["top_k"])
        bufs = [self._x(x) for x in experts]
        key = ("ptrs", t.id)
        ptrs = self._moe_ptrs.get(key)
        if ptrs is None and self.gpu:
            ptrs = torch.tensor([b.data_ptr() for b in bufs], dtype=torch.int64, device=self.device)
            self._moe_ptrs[key] = ptrs
        ops.moe_gather_combine(bufs, idx, slot, off, gate, residual=self._x(res_name), out=out, ptrs=ptrs,
                               post_norm=self._post_norm_out(self._flat(out)))

    def _attn_block_ok(self, head: Task, norm: Optional[Task], x, residual, out, B: int, S: int) -> bool:
        """Can this attention group run as the one-launch block (ops.attn_block)? GPU, MHA with
        head_dim 64, no RoPE, causal, a norm folded with row statistics handed over by x's
        producer, the residual in the group, no post-norm of the output, a shape the kernel
        takes, and a weight no other reader shares."""
        a, W = head.op.attrs, head.op.weights
        if not (self.gpu and ATTN_BLOCK) or norm is None or residual is None or a.get("rope") \
                or not a.get("causal", True) or a["n_kv_head"] != a["n_head"]:
            return False
        if self._ext_stats.get(norm.op.inputs[0]) is None or x.shape[-1] > FOLD_MAX_K \
                or self._pn_given == norm.id or self._pn is not None:
            return False
        if self._w_users.get(W["w_qkv"], 1) > 1:
            return False
        return ops.attn_block_ok(x.shape[0], x.shape[-1], B, S, a["n_head"], a["n_kv_head"], a["head_dim"])

    def _run_group(self, ins) -> None:
        grp = [self.tasks[t] for t in ins.group]
        norm = None
        if len(grp) > 1 and grp[0].op.kind in ("layernorm", "rmsnorm"):
            norm, grp = grp[0], grp[1:]
        head, tail = grp[0], grp[-1]
        out = self._views[tail.id]
        k = head.op.kind
        residual = None
        if tail.op.kind == "residual" and len(grp) > 1:
            prod = grp[-2].id
            other = [d for d in tail.op.inputs if d != prod][0]
            residual = self._flat(self._x(other))
        act = "gelu" if any(t.op.kind == "gelu" for t in grp[1:]) else head.op.attrs.get("act")
        st_out = self._stats_out.get(tail.id)  # this group's output feeds a folded norm: emit row stats
        a = head.op.attrs
        W = head.op.weights
        src = norm.op.inputs[0] if norm is not None else (head.op.inputs[0] if head.op.inputs else None)
        if k == "embedding":
            tok = self._x(head.op.inputs[0])
            B, S = head.op.out_shape[0], head.op.out_shape[1]
            wpe = self._w(W["wpe"]) if "wpe" in W else None
            if "seq_chunk" in a:  # sequence chunk c: its token slice, positions from c*S on
                c, P = a["seq_chunk"]
                tok = tok.view(B, S * P)[:, c * S:(c + 1) * S]
                tok = tok.reshape(-1) if B == 1 else tok.contiguous().view(-1)
                if wpe is not None:
                    wpe = wpe[c * S:(c + 1) * S]
            zero = self._stats_slab if (self._zero_in_embedding and ins is self._zero_run) else None
            if st_out is not None and zero is not None:
                if st_out.data_ptr() != zero.data_ptr():
                    raise RuntimeError("an embedding's row statistics must lead the statistics slab")
                zero = zero[st_out.numel():]
            ops.embedding(tok, self._w(W["wte"]), wpe, S, out=self._flat(out), zero=zero, stats=st_out)
        elif k in ("layernorm", "rmsnorm") and self._pn_given == head.id:
            pass  # written by the producer of its input (_plan_post_norm)
        elif k == "layernorm":
            ops.layernorm(self._flat(self._x(src)), self._w(W["w"]), self._w(W["b"]), a.get("eps", 1e-5),
                          out=self._flat(out))
        elif k == "rmsnorm":
            ops.rmsnorm(self._flat(self._x(src)), self._w(W["w"]), a.get("eps", 1e-5), out=self._flat(out))
        elif k == "residual":
            ops.add(self._x(head.op.inputs[0]), self._x(head.op.inputs[1]), out=out)
        elif k == "gelu":
            ops.gelu(self._x(src), out=out)
        elif k == "linear" and head.id in self._gate_route and norm is None and residual is None \
                and st_out is None and "b" not in W and not act:
            # router of a batched MoE layer: logits + top-k + expert-sorted order in one launch,
            # memoised for the layer's experts and combine (_moe_route)
            E, K = self._gate_route[head.id]
            self._moe_memo[("route", head.id)] = ops.moe_gate_route(self._flat(self._x(src)), self._w(W["w"]), K,
                                                                    self._flat(out))
        elif k in ("linear", "lm_head"):
            self._gemm(self._flat(self._x(src)), W["w"], W.get("b"), norm, act=act, residual=residual,
                       out=self._flat(out), stats_out=st_out)
        elif k == "attention":
            x = self._flat(self._x(src))
            M = x.shape[0]
            B, S = head.op.out_shape[0], head.op.out_shape[1]
            nh, nkv, D = a["n_head"], a["n_kv_head"], a["head_dim"]
            width = (nh + 2 * nkv) * D
            qkv = self._ws(0, (M, width))
            o = self._ws(M * width, (M, nh * D))
            if self._attn_block_ok(head, norm, x, residual, out, B, S):
                W1, cs, bd = self._prep(W["w_qkv"], norm, W.get("b_qkv"))
                if self._attn_sync is None:  # (first, eager step: never allocated during capture)
                    self._attn_sync = ops.attn_block_sync(M, S, B, nh, self.device)
                ops.attn_block(x, W1, bd, cs, self._ext_stats[norm.op.inputs[0]], norm.op.kind,
                               norm.op.attrs.get("eps", 1e-5), qkv, o, self._w(W["w_o"]),
                               self._w(W["b_o"]) if "b_o" in W else None, residual, self._flat(out), B, S, nh,
                               stats_out=st_out, sync=self._attn_sync)
                return
            if a.get("rope"):
                # RoPE in the QKV GEMM epilogue (q/k rows pair-interleaved at load time)
                cos, sin = self._rope_tables(S, D, a.get("rope_theta", 10000.0))
                self._gemm(x, W["w_qkv"], W.get("b_qkv"), norm, out=qkv, rope=(cos, sin, S, D, (nh + nkv) * D),
                           rope_perm=(nh, nkv, D))
            else:
                self._gemm(x, W["w_qkv"], W.get("b_qkv"), norm, out=qkv)
            ops.attention(qkv[:, :nh * D], qkv[:, nh * D:(nh + nkv) * D], qkv[:, (nh + nkv) * D:], B, S, nh, nkv,
                          D, causal=a.get("causal", True), out=o)
            ops.linear(o, self._w(W["w_o"]), self._w(W["b_o"]) if "b_o" in W else None, residual=residual,
                       out=self._flat(out), stats_out=st_out, post_norm=self._post_norm_out(self._flat(out)))
        elif k == "qkv_proj":
            # sequence chunk c's QKV rows (RoPE at its absolute positions c*Sc ..)
            x = self._flat(self._x(src))
            B, Sc = head.op.out_shape[0], head.op.out_shape[1]
            nh, nkv, D = a["n_head"], a["n_kv_head"], a["head_dim"]
            c, P = a["seq_chunk"]
            if a.get("rope"):
                cos, sin = self._rope_tables(Sc * P, D, a.get("rope_theta", 10000.0))
                self._gemm(x, W["w_qkv"], W.get("b_qkv"), norm, out=self._flat(out),
                           rope=(cos[c * Sc:], sin[c * Sc:], Sc, D, (nh + nkv) * D), rope_perm=(nh, nkv, D))
            else:
                self._gemm(x, W["w_qkv"], W.get("b_qkv"), norm, out=self._flat(out))
        elif k == "attn_sp":
            B, Sc = head.op.out_shape[0], head.op.out_shape[1]
            nh, nkv, D = a["n_head"], a["n_kv_head"], a["head_dim"]
            c, P = a["seq_chunk"]
            M = B * Sc
            chunks = [self._flat(self._x(n)) for n in head.op.inputs]  # qkv of the visible chunks
            q = chunks[c][:, :nh * D]
            nkeys = len(chunks) * Sc
            if len(chunks) == 1:
                kv = chunks[0][:, nh * D:]
            else:  # gather the chunks' K/V rows into one [B, keys, 2*nkv*D] block
                kv = self._ws(0, (B, nkeys, 2 * nkv * D))
                for j, ch in enumerate(chunks):
                    kv[:, j * Sc:(j + 1) * Sc].copy_(ch.view(B, Sc, -1)[:, :, nh * D:])
                kv = kv.view(B * nkeys, 2 * nkv * D)
            o = self._ws(2 * B * nkeys * 2 * nkv * D // 2 + 256, (M, nh * D))
            ops.attention(q, kv[:, :nkv * D], kv[:, nkv * D:], B, nkeys, nh, nkv, D,
                          causal=a.get("causal", True), out=o, Sq=Sc, q_off=c * Sc)
            ops.linear(o, self._w(W["w_o"]), self._w(W["b_o"]) if "b_o" in W else None, residual=residual,
                       out=self._flat(out), stats_out=st_out)
        elif k == "swiglu_mlp":
            x = self._flat(self._x(src))
            M, F = x.shape[0], a["ffn"]
            h = self._ws(0, (M, F))
            self._gemm(x, W["w_gate_up"], None, norm, act="swiglu", out=h)  # SwiGLU in the epilogue
            ops.linear(h, self._w(W["w_down"]), residual=residual, out=self._flat(out), stats_out=st_out,
                       post_norm=self._post_norm_out(self._flat(out)))
        elif k == "moe_expert":
            self._moe_expert(head, self._flat(out))
        elif k == "moe_combine":
            self._moe_combine(head, self._flat(out))
        elif k == "sum":
            # tensor-parallel shard partials
            ins_ = head.op.inputs
            acc = self._x(ins_[-1])
            for name in ins_[:-1]:
                ops.add(self._x(name), acc, out=out)
                acc = out
        else:
            raise NotImplementedError(f"op kind {k!r}")

    # ------------------------------------------------------------------- step
    def _mark(self):
        """A timestamp token: a recorded hipEvent on GPU, host time on the CPU backend."""
        if self.gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def _step_body(self, stats: StepStats, events: Optional[list] = None) -> None:
        """Issue the program. ``events`` (profiling) collects (name, category, t0, t1) tokens."""
        _tuning.set_model(self.model_name)
        tr = self.trace
        self._pending_sends = {}
        self._reset_step_state()
        if self._device_p2p:
            self.comm.begin_step()  # this rank's step counter: the sequence number of its flags
        if self._rec is not None and not self.gpu:  # replayed steps reset it too
            self._rec.r.add_pycall(self._reset_step_state)
        if self.prog.start_resident:  # warm-started program: its start groups are resident
            first = not self._started
            for pid, off in self.prog.start_resident.items():
                o, total, layout, views = self._views_at(off, pid)
                if first:  # one-time fill before the first step
                    self._fill(o, total, layout, views, pid, stats)
                self._map(pid, o, total, views)
        self._started = True
        if self._stats_slab is not None and not self._zero_in_embedding:
            if self._rec is not None:
                self._rec.r.add_memset(self._stats_slab, 0, 0)
            else:
                self._stats_slab.zero_()

        recv_work: Dict[str, Tuple[object, object]] = {}
        hoist = self._hoist if self._copy_stream is not None else None
        pending: Dict[int, object] = {}
        if hoist:
            pending, self._carry = self._carry, {}  # issued by the previous step's tail
            if self._rec is not None:  # those fills: the runner's cross-step events
                pending = {k: (None if v is None else self._rec.event(carry_load=k)) for k, v in pending.items()}
        if hoist and -1 in hoist and any(k not in pending for k in hoist[-1]):
            ev0 = self._new_event()
            self._record(ev0)
            for k in hoist[-1]:
                if k not in pending:
                    self._prefetch(k, ev0, stats, pending, events)
        segs = self._segments if (events is None and not tr) else {}
        pulls = sorted(self._pull_at)
        n_ins = len(self.prog.instrs)
        i = -1
        while i + 1 < n_ins:
            i += 1
            ins = self.prog.instrs[i]
            seg_end = None
            if ins.op == "run" and (i in segs or (self._capture_plan and i in self._capture_plan)):
                seg_end = segs[i][0] if i in segs else self._capture_plan[i]
                for k in range(i, seg_end):  # everything the segment's runs wait for, before it
                    self._pre_run(self.prog.instrs[k], recv_work, events)
                if i in segs:
                    if segs[i][1] is None:
                        pass  # an empty segment (its runs were folded into other launches)
                    elif self._rec is not None:
                        self._rec.r.add_graph(segs[i][1].raw_cuda_graph_exec())
                    else:
                        segs[i][1].replay()
                else:  # capture_segments: record this segment's kernels
                    self._segments[i] = (seg_end, self._capture_segment(i, seg_end, stats))
                stats.kernels += seg_end - i
                i = seg_end - 1
                ins = self.prog.instrs[i]
            if tr:
                Roctx.push(f"{ins.op}:{ins.task or ins.param}")
            if seg_end is not None:
                pass
            elif ins.op == "psend":
                self._psend(i, ins, stats)
            elif ins.op == "load" and ins.peer >= 0 and self._steps_done > 0:
                self._peer_load(i, ins, stats)
            elif ins.op == "load" and hoist is not None and i in pending:
                off, total, layout, views = self._group_views(i, ins.param)
                self._map(ins.param, off, total, views)
                done = pending.pop(i)
                if done is not None:  # the compute stream waits at the group's first reader
                    self._await[ins.param] = done
            elif ins.op == "load":
                self._wait_sends(ins)  # the region may still be read by a parameter send
                t0 = self._mark() if events is not None else None
                fills = stats.param_fills
                self._load(i, ins.param, stats)
                if events is not None and stats.param_fills != fills:
                    events.append((ins.param, "load", t0, self._mark()))
            elif ins.op == "evict":
                self._await_fill(ins.param)
                self._evict(ins.param)
            elif ins.op in ("send", "recv"):
                # every send / recv posted at this program point: ONE p2p group
                # (a recv whose buffer is still being sent by a send of the same group starts a
                # new group: that send must complete before the recv is posted)
                j = i
                while j + 1 < n_ins and self.prog.instrs[j + 1].op in ("send", "recv") \
                        and not any(i <= w <= j for w in self.prog.instrs[j + 1].wait_sends) \
                        and not (hoist and (j in hoist or j in self._carry_at)) and not tr:
                    j += 1
                self._post_p2p(i, j + 1, recv_work, stats, events)
                i = j
                ins = self.prog.instrs[i]
            elif ins.op == "run":
                self._pre_run(ins, recv_work, events)
                if self._rec is not None:  # CPU runner: the group runs as a callback, with the
                    # parameter mapping of this point of the step (a GPU segment has its pointers baked in)
                    snap = (dict(self._params), dict(self._wflat), dict(self._region), list(self._valid))
                    self._rec.r.add_pycall(lambda _i=i, _ins=ins, _s=snap: self._run_snapshot(_i, _ins, _s))
                else:
                    self._issue_run(i, ins, stats, events)
                stats.kernels += 1
            while pulls and pulls[0] <= i:  # routed hidden rows whose router logits are here now
                for h in self._pull_at[pulls.pop(0)]:
                    self._pull_hidden_rows(h)
            if hoist and i in self._carry_at:  # the next step's first refills, under this tail
                evc = self._new_event()
                self._record(evc)
                for k in self._carry_at[i]:
                    self._prefetch(k, evc, stats, self._carry, events, carry=True)
            if hoist and i in hoist:  # loads whose region is free from here on
                ev = self._new_event()
                self._record(ev)
                for k in hoist[i]:
                    self._prefetch(k, ev, stats, pending, events)
            if tr:
                Roctx.pop()
        for done in pending.values():  # (none in a well-formed program: each load is reached)
            if done is not None:
                self._stream_wait(torch.cuda.current_stream(self.device), done)
        for pid in list(self._await):
            self._await_fill(pid)
        for w, _ in recv_work.values():
            w.wait()
        for w in self._deferred.values():  # (a routed receive no MoE node took: the whole region)
            w.wait()
        self._deferred = {}
        for w in self._pending_sends.values():
            w.wait()
        self._pending_sends = {}
        for w in self._param_recv.values():
            w.wait()
        self._param_recv = {}
        self._steps_done += 1

    def _post_p2p(self, a: int, b: int, recv_work, stats: StepStats, events) -> None:
        """Instructions [a, b) (sends and recvs) posted as one group."""
        ops_, idx = [], []
        for k in range(a, b):
            ins = self.prog.instrs[k]
            if ins.op == "recv":
                self._wait_sends(ins)  # the recv buffer may still be read by a send to another peer
            buf = self._act_region(ins.task) if self._device_p2p else self._ep_buf(ins, self._views[ins.task])
            ops_.append((ins.op == "send", buf, ins.peer, ("act", ins.task)))
            idx.append(k)
        t0 = self._mark() if events is not None else None
        works = self._p2p_group(ops_)
        for k, (snd, buf, peer, _), w in zip(idx, ops_, works):
            ins = self.prog.instrs[k]
            nbytes = buf.numel() * buf.element_size()
            if snd:
                self._pending_sends[k] = w
                if events is not None:
                    events.append((f"{ins.task}->gpu{peer}", "send", t0, self._mark()))
                stats.sends += 1
                stats.bytes_sent += nbytes
            else:
                stats.recvs += 1
                stats.bytes_recv += nbytes
                if self._device_p2p and ins.task in self._routed_out:
                    self._pull_expert_rows(ins.task, w)  # the home's routing is known: pull now
                elif self._device_p2p and ins.task in self._routed_in:
                    self._deferred[ins.task] = w  # pulled once its router logits are here (_pull_at)
                else:
                    if self._device_p2p:
                        # pulled HERE, at the producer's position, as an RCCL receive completes once
                        # both ends posted: a pull deferred to the consumer could wait for a peer that
                        # is itself waiting for this rank to release the source (its ack comes with
                        # the pull); each after its own flag, in order (one wait for all: validate.py)
                        w.wait()
                    recv_work[ins.task] = (w, t0)
                if self._device_p2p:  # hidden states whose router logits just came: right away
                    for h in self._pull_at.get(k, ()):
                        self._pull_hidden_rows(h)

    def _run_snapshot(self, i, ins, snap) -> None:
        self._params, self._wflat, self._region, self._valid = (dict(snap[0]), dict(snap[1]), dict(snap[2]),
                                                                list(snap[3]))
        self._issue_run(i, ins, StepStats(), None)

    def _reset_step_state(self) -> None:
        self._moe_memo = {}
        self._pn_done = None
        self._deferred = {}

    def _pull_expert_rows(self, x: str, w) -> None:
        """An expert's compact output rows, pulled at their post: the home's routing of the layer
        is known there, so only the expert's count of rows crosses — and the producer's ack comes
        as early as an RCCL receive's completion (a pull left to the combine could keep a peer
        waiting for its region while this rank waits for one of that peer's)."""
        t = self.tasks[x]
        off = self._moe_route(t.op.inputs[1], t.op.attrs["n_experts"], t.op.attrs["top_k"])[4]
        v = self._views[x]
        M, H = math.prod(v.shape[:-1]), v.shape[-1]
        w.pull_rows(self._act_region(x), H * v.element_size(), None, off, self._exp_ids[x], M)

    def _pull_hidden_rows(self, h: str) -> None:
        """A received hidden state's routed rows, pulled right after its router logits are on
        this rank (``_pull_at``): into the cross-request batch's block when its experts run as
        one (co-run span), else into the request's own buffer."""
        if h not in self._deferred:
            return
        r, E, K = self._h_route[h]
        blk = self._xblock.get(h)
        out = None
        if blk is not None:
            q, R, H = blk
            out = self._scratch("moe_xpb", self._xpb_shape)[q * R:(q + 1) * R]
        self._moe_permuted(h, r, E, K, out=out)

    def _plan_routed_edges(self) -> None:
        """Expert-parallel edges that move ROUTED ROWS only (device transport): a hidden state
        received here whose every local consumer is an expert node reading it as its tokens, and
        an expert's output received here whose consumer is the layer's combine. Only the rows the
        local experts were routed move (gathered into the expert-sorted order), and only an
        expert's count of compact output rows: bytes = routed rows, no capacity, no host sync.
        Each is pulled as soon as the device-side routing it needs is on this rank — an expert
        output at its post (the home's own routing), a hidden state right after its router
        logits arrived (``_pull_at``) — so its producer's ack never waits for a later consumer
        (the device analogue of RCCL's completion once both ends posted)."""
        from .program import device_routed_edges

        self._h_route: Dict[str, Tuple[str, int, int]] = {}
        routed_in, routed_out = device_routed_edges(self.prog, self.tasks, self._moe_batched_ids)
        for x, us in routed_in.items():
            ex = sorted({u.op.attrs["expert"] for u in us})
            self._routed_in[x] = torch.tensor(ex, dtype=torch.int32, device=self.device)
            u = us[0]
            self._h_route[x] = (u.op.inputs[1], u.op.attrs["n_experts"], u.op.attrs["top_k"])
        for x in routed_out:
            self._routed_out.add(x)
            self._exp_ids[x] = torch.tensor([self.tasks[x].op.attrs["expert"]], dtype=torch.int32, device=self.device)
        at: Dict[str, int] = {}  # where each tensor is on this rank: its run, or its receive
        for i, ins in enumerate(self.prog.instrs):
            if ins.op == "run":
                for tid in ins.group:
                    at.setdefault(tid, i)
            elif ins.op == "recv":
                at.setdefault(ins.task, i)
        for h, (r, _, _) in self._h_route.items():
            self._pull_at.setdefault(max(at[h], at[r]), []).append(h)

    # ------------------------------------------------- expert-parallel capacity edges (RCCL)
    def _plan_ep_capacity(self) -> None:
        """Expert-parallel edges as fixed-capacity messages on the RCCL / hub / gloo transports
        (program.plan_ep_capacity sets ``Instr.rows``): the home rank packs the rows its routing
        sends to an expert GPU right after the router runs (ops.moe_pack, inside the step's
        kernels: no host sync), sends ``rows`` rows; the expert GPU unpacks them into the
        expert-sorted layout its experts read; an expert's compact output returns in ``erows``
        rows. A capacity GROUP is one (hidden state, other rank) pair — the hidden edge and its
        experts' return edges; both of its ranks compute the same counts from the same router
        logits, so both see an overflow (``ep_overflow``) and widen the same group."""
        self._ep_groups: Dict[Tuple[str, int], int] = {}  # (tokens tensor, other rank) -> flag index
        self._ep_full: set = set()                          # widened groups: whole-buffer edges
        self._ep_msg: Dict[Tuple[str, int], Tuple[int, Tuple[str, int]]] = {}  # (task, peer) -> (rows, group)
        self._ep_pack_at: Dict[str, List[tuple]] = {}       # router -> [(h, dst, experts, rows, erows)]
        self._ep_unpack: Dict[str, tuple] = {}              # received h -> (src, experts, rows, erows)
        self._ep_route: Dict[str, Tuple[str, int, int]] = {}  # h -> (router, E, top-k)
        self._ep_bufs: Dict[Tuple[str, int], torch.Tensor] = {}
        self._ep_ovf: Optional[torch.Tensor] = None
        if self._device_p2p or self.comm is None:
            return  # (the device transport pulls exactly the routed rows: _plan_routed_edges)
        for t in self.tasks.values():
            if t.op is not None and t.op.kind == "moe_expert":
                self._ep_route.setdefault(t.op.inputs[0], (t.op.inputs[1], t.op.attrs["n_experts"],
                                                           t.op.attrs["top_k"]))
        for ins in self.prog.instrs:
            if ins.op in ("send", "recv") and ins.rows and ins.experts:
                g = (ins.task, ins.peer)
                self._ep_groups.setdefault(g, len(self._ep_groups))
                self._ep_msg[g] = (ins.rows, g)
                if ins.op == "send":
                    r = self._ep_route[ins.task][0]
                    self._ep_pack_at.setdefault(r, []).append((ins.task, ins.peer, ins.experts, ins.rows, ins.erows))
                else:
                    self._ep_unpack[ins.task] = (ins.peer, ins.experts, ins.rows, ins.erows)
        for ins in self.prog.instrs:  # return edges: grouped with their tokens' edge
            if ins.op in ("send", "recv") and ins.rows and not ins.experts:
                g = (self.tasks[ins.task].op.inputs[0], ins.peer)
                if g not in self._ep_groups:
                    raise RuntimeError(f"rank {self.prog.rank}: capacity edge {ins.task} without its tokens' edge")
                self._ep_msg[(ins.task, ins.peer)] = (ins.rows, g)
        if self._ep_groups:
            self._ep_ovf = torch.zeros(len(self._ep_groups), dtype=torch.int32, device=self.device)

    def _ep_buf(self, ins, buf):
        """The message of a send / recv: its capacity rows unless its group was widened."""
        m = self._ep_msg.get((ins.task, ins.peer))
        if m is None or m[1] in self._ep_full:
            return buf
        rows = m[0]
        if ins.op == "send" and ins.experts:  # packed at the router's run (_ep_pack)
            return self._ep_bufs[(ins.task, ins.peer)][:rows]
        return self._flat(buf)[:rows]

    def _ep_pack(self, r: str) -> None:
        """Right after the router ``r`` ran on the home rank: pack, for every expert GPU with a
        capacity edge of this layer, the token rows routed to its experts (one launch)."""
        dests = []
        for h, dst, experts, rows, erows in self._ep_pack_at[r]:
            g = (h, dst)
            if g in self._ep_full:
                continue
            buf = self._ep_bufs.get(g)
            if buf is None:  # (first, eager step: never allocated during capture)
                H = self.tasks[h].op.out_shape[-1]
                buf = self._ep_bufs[g] = torch.empty(rows, H, dtype=self.dtype, device=self.device)
            f = self._ep_groups[g]
            dests.append((h, (buf, rows, experts, f, [erows] * len(experts), [f] * len(experts))))
        if not dests:
            return
        _, E, K = self._ep_route[dests[0][0]]
        route = self._moe_route(r, E, K)
        for h in dict.fromkeys(d[0] for d in dests):
            ds = [d for hh, d in dests if hh == h]
            for k in range(0, len(ds), 8):  # kMoePackMaxDest
                ops.moe_pack(self._flat(self._x(h)), route[2], route[4], ds[k:k + 8], self._ep_ovf)

    def ep_overflow(self) -> List[Tuple[str, int]]:
        """Capacity groups whose routing exceeded a capacity since the last widening (a host read:
        synchronises). Those steps' MoE outputs are wrong for the rows that did not fit."""
        if self._ep_ovf is None:
            return []
        flags = self._ep_ovf.tolist()
        return [g for g, i in self._ep_groups.items() if flags[i] and g not in self._ep_full]

    def widen_ep(self, groups) -> None:
        """Carry these capacity groups as whole buffers from now on (exact for any routing). The
        captured graphs bake message sizes in: they are dropped (call ``capture`` again)."""
        groups = [g for g in groups if g in self._ep_groups]
        if not groups:
            return
        self._ep_full |= set(groups)
        self._ep_ovf.zero_()
        self._segments, self._graph, self._graph_exec, self._fast = {}, None, None, None
        self._drop_runner()

    def _pre_run(self, ins, recv_work, events) -> None:
        """What a run must wait for: copy-stream fills and peer receives of its parameter
        groups, receives of its inputs, in-flight sends of the region it overwrites — for a
        co-run span's first run, what every member waits for (they all run there)."""
        span = self._xfirst.get(ins.task) if ins.op == "run" else None
        for x in ([self.prog.instrs[k] for k in span] if span else [ins]):
            self._pre_run_one(x, recv_work, events)

    def _pre_run_one(self, ins, recv_work, events) -> None:
        for tid in ins.group:
            for pid in self.tasks[tid].params_needed:
                self._await_fill(pid)
                pw = self._param_recv.pop(pid, None)
                if pw is not None:
                    pw.wait()  # the group arrives from a peer's HBM
            for d in self.tasks[tid].dependencies:
                rw = recv_work.pop(d, None)
                if rw is not None:
                    if d in self._routed_in or d in self._routed_out:
                        self._deferred[d] = rw[0]  # routed rows, pulled by the MoE code
                        continue
                    rw[0].wait()
                    if events is not None:
                        events.append((d, "recv", rw[1], self._mark()))
        self._wait_sends(ins)  # output region about to be overwritten: its sends must be done

    def _issue_run(self, i: int, ins, stats: StepStats, events) -> None:
        given = self._norm_given.get(i)
        self._pn, self._pn_given = self._post_norm.get(i), (given if given == self._pn_done else None)
        if given is not None:
            self._pn_done = None
        try:
            self._issue_run_body(i, ins, stats, events)
        finally:
            self._pn = self._pn_given = None

    def _issue_run_body(self, i: int, ins, stats: StepStats, events) -> None:
        run = self._run_group
        if i in self._moe_batch:  # the layer's experts in one grouped launch pair
            run = lambda _ins, _i=i: self._run_moe_batch(_i, stats)  # noqa: E731
        elif i in self._xbatch:  # the layer's experts here over every request: one launch pair
            run = lambda _ins, _i=i: self._run_moe_xbatch(_i, stats)  # noqa: E731
        elif i in self._moe_skip or i in self._mlp_skip or i in self._xskip:  # ran with a batch / MLP block
            run = None
        elif i in self._mlp_fused:  # fc1 + fc2 of the MLP block in one launch
            run = lambda _ins, _i=i: self._run_mlp_fused(_i)  # noqa: E731
        if run is not None and events is not None:
            t0 = self._mark()
            run(ins)
            events.append((ins.task, "kernel", t0, self._mark()))
        elif run is not None:
            run(ins)
        if self._ep_pack_at and run is not None:  # a router whose rows leave through capacity edges
            for tid in ins.group:
                if tid in self._ep_pack_at:
                    self._ep_pack(tid)

    def _psend(self, i: int, ins, stats: StepStats) -> None:
        """Send a resident parameter group to a peer that re-fills it from this rank's HBM
        (program.plan_peer_fills). The first step has no parameter transfers: every rank fills
        from its host image and applies its kernels' in-place weight transforms first."""
        if self._steps_done == 0:
            return
        self._await_fill(ins.param)
        pw = self._param_recv.pop(ins.param, None)
        if pw is not None:
            pw.wait()  # this rank received the group itself: forward it once it arrived
        total = group_layout(self.store.groups[ins.param])[0]
        buf = self.param_slab[ins.param_off:ins.param_off + total]
        self._pending_sends[i] = self._isend(buf, ins.peer, ("param", ins.param, ins.gpos))
        stats.sends += 1
        stats.bytes_sent += total

    def _peer_load(self, i: int, ins, stats: StepStats) -> None:
        """Load a parameter group by receiving it from the peer that holds it."""
        self._wait_sends(ins)
        off, total, layout, views = self._group_views(i, ins.param)
        self._overwrite(off, total, ins.param)
        self._map(ins.param, off, total, views)
        for spec, _ in layout:
            if spec.name not in self._derived_named:
                self._derived_cache.pop((spec.name, views[spec.name].data_ptr()), None)
                self._derived_cache.pop(("side", spec.name, views[spec.name].data_ptr()), None)
        self._param_recv[ins.param] = self._irecv(self.param_slab[off:off + total], ins.peer,
                                                  ("param", ins.param, ins.gpos))
        if self._device_p2p:
            self._param_recv[ins.param].wait()  # pulled at the message's position (see _post_p2p)
        self._valid.append((off, total, ins.param))
        stats.recvs += 1
        stats.peer_fills += 1
        stats.bytes_peer += total

    def _wait_sends(self, ins) -> None:
        """Complete the in-flight sends whose buffer ``ins`` is about to overwrite (planned
        statically: Instr.wait_sends, program._plan_send_waits)."""
        for j in ins.wait_sends:
            w = self._pending_sends.pop(j, None)
            if w is not None:
                w.wait()

    def step(self, profile: bool = False) -> StepStats:
        """Execute the rank's program once (asynchronously on the GPU). ``profile=True`` runs
        it eagerly with a timestamp pair around every instruction and fills
        ``stats.timeline`` (kernel groups) and ``stats.events`` (kernels, parameter fills,
        p2p sends/recvs), in ms from the step start."""
        if self._fast is not None and not profile:  # a captured whole step: one graph launch
            self._fast[0](self._fast[1], self._fast[2])
            if self._mlp_fused:
                self.check_mlp_fused()
            if self._fast[4]:
                self._watch()
            self.last = self._fast[3]
            return self._fast[3]
        stats = StepStats()
        if self._runner is not None and profile:
            self._leave_runner()
        if self._runner is not None:
            if self.trace:
                Roctx.push(f"runner_step:rank{self.prog.rank}")
            self._runner.run()
            if self.trace:
                Roctx.pop()
            stats = StepStats(**{k: getattr(self._runner_stats, k) for k in ("kernels", "sends", "recvs",
                                                                              "bytes_sent", "bytes_recv",
                                                                              "param_fills", "bytes_filled",
                                                                              "peer_fills", "bytes_peer")})
        elif self._graph is not None and not profile:
            if self.trace:
                Roctx.push(f"graph_step:rank{self.prog.rank}")
            if self._graph_exec is not None:  # GIL released
                ops.ext().graph_launch(self._graph_exec, torch.cuda.current_stream(self.device).cuda_stream)
            else:
                self._graph.replay()
            if self.trace:
                Roctx.pop()
            stats.kernels = self.prog.n_kernels
        else:
            ev = [] if profile else None
            t_begin = self._mark() if profile else None
            self._step_body(stats, ev)
            if ev is not None:
                if self.gpu:
                    self._sync()
                    el = lambda a: t_begin.elapsed_time(a)  # noqa: E731
                else:
                    el = lambda a: (a - t_begin) * 1e3  # noqa: E731
                stats.events = [(n, c, el(a), el(b)) for n, c, a, b in ev]
                stats.timeline = [(n, a, b) for n, c, a, b in stats.events if c == "kernel"]
        if self._mlp_fused:
            self.check_mlp_fused()
        if self._device_p2p or self._attn_sync is not None:
            self._watch()
        if self.debug:
            self.check_guards()
        self.last = stats
        return stats

    # ------------------------------------------------------------ device-transport health
    def transport_errors(self) -> int:
        """This rank's device-transport error word (bit 0: a pull, bit 1: an ack wait timed
        out); 0 for RCCL / the loopback hub. A host read (synchronises on the GPU)."""
        return int(self.comm.errors()) if self._device_p2p and not self.comm.dry else 0

    def check_transport(self) -> None:
        """Raise :class:`TransportError` (naming the rank and the edges still behind) if any
        device-transport wait of this rank gave up since the last reset."""
        err = self.transport_errors()
        if err:
            raise TransportError(self._transport_msg(err))

    def reset_transport_errors(self) -> None:
        """Clear the error word and its host mirror (after warm-up: a cold first step's
        code-object loading on one rank can outlast a peer's wait)."""
        if self._device_p2p:
            self.comm.reset_errors()
            if self._err_mirror is not None:
                self._err_mirror.zero_()

    def _transport_msg(self, err: int) -> str:
        from .devp2p import ERR_ACK, ERR_PULL, TIMEOUT_S

        what = [n for bit, n in ((ERR_PULL, "a pull"), (ERR_ACK, "an ack wait")) if err & bit]
        behind = self.comm.stalled() if hasattr(self.comm, "stalled") else []
        msg = (f"rank {self.prog.rank}: device transport: {' and '.join(what) or 'a wait'} timed out "
               f"(error word {err}, DLS_P2P_TIMEOUT_S={TIMEOUT_S}); this rank's outputs are wrong")
        if behind:
            msg += "; edges behind: " + "; ".join(behind[:8]) + (" ..." if len(behind) > 8 else "")
        return msg

    def _watch(self) -> None:
        """After a step is issued: every P2P_CHECK_EVERY-th step read the host mirrors of the
        device error words — the device transport's, and the one-launch attention blocks' —
        (written by asynchronous copies issued at the previous check, behind that step's kernels)
        and issue the next copies: a wait that gave up fails a later step loudly without a host
        synchronisation per step. The host transport (CPU) reads its word directly, every step."""
        p2p = self._device_p2p and not self.comm.dry
        if p2p and not self.gpu:
            err = self.comm.errors()
            if err:
                raise TransportError(self._transport_msg(err))
            p2p = False
        if not self.gpu or not (p2p or self._attn_sync is not None):
            return
        self._watch_n += 1
        if self._watch_n % P2P_CHECK_EVERY:
            return
        if p2p:
            m = self._err_mirror
            if m is None:
                m = self._err_mirror = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            seen = int(m[0])
            if seen:
                raise TransportError(self._transport_msg(seen))
            m.copy_(self.comm.mb.err, non_blocking=True)
        if self._attn_sync is not None:
            m = self._attn_mirror
            if m is None:
                m = self._attn_mirror = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            if int(m[0]):
                raise RuntimeError(self._attn_msg())
            m.copy_(self._attn_sync[-1:], non_blocking=True)

    def _attn_msg(self) -> str:
        return (f"rank {self.prog.rank}: a one-launch attention block (ops.attn_block) gave up waiting for its "
                f"q/k/v or attention tiles; the step's outputs are wrong")

    def check_attn_block(self) -> None:
        """Synchronous read of the one-launch attention blocks' error word (raises if set)."""
        if self._attn_sync is not None and int(self._attn_sync[-1].item()) != 0:
            raise RuntimeError(self._attn_msg())

    def check_mlp_fused(self) -> None:
        """The one-launch MLP block (DLS_MLP_FUSED=1, off by default) gives up a poll after its
        spin limit and proceeds with wrong numbers rather than hang; its error word is read here
        after every step (a host synchronisation: the price of the opt-in path) and a set word
        fails the step loudly."""
        if self._mlp_sync is not None and int(self._mlp_sync[-1].item()) != 0:
            raise RuntimeError(f"rank {self.prog.rank}: fused MLP block gave up waiting for fc1 tiles "
                               f"(error word {int(self._mlp_sync[-1].item())}); this step's outputs are wrong")

    def check_guards(self) -> None:
        """Debug mode: every arena's trailing canary is intact and the rank's outputs are
        finite (a kernel writing past its planned region or producing NaN fails loudly)."""
        if self.gpu:
            self._sync()
        for name, full in (("activation", self._act_full), ("parameter", self._param_full),
                           ("workspace", self._ws_full)):
            tail = full[-GUARD_BYTES:]
            if not bool((tail == GUARD_VALUE).all()):
                raise RuntimeError(f"rank {self.prog.rank}: {name} arena guard overwritten (out-of-bounds write)")
        for ins in self.prog.instrs:
            if ins.op == "run" and not self._consumed_locally(ins.task):
                v = self._views[ins.task]
                if not bool(torch.isfinite(v.float()).all()):
                    raise RuntimeError(f"rank {self.prog.rank}: non-finite values in output of {ins.task}")

    def _consumed_locally(self, tid: str) -> bool:
        """True if ``tid`` is read by a later group on this rank or sent away (its buffer may
        legitimately be reused afterwards, so only final outputs are checked)."""
        if self._local_consumed is None:
            used = set()
            for ins in self.prog.instrs:
                if ins.op == "run":
                    for t in ins.group:
                        used.update(self.tasks[t].dependencies)
                elif ins.op == "send":
                    used.add(ins.task)
            self._local_consumed = used
        return tid in self._local_consumed

    def capture(self) -> bool:
        """Capture the steady-state step into a hipGraph: the whole step for a comm-free
        program without copy-stream refills, else its kernel-group segments (capture_segments)."""
        if not self.use_graph:
            return False
        self._drop_runner()  # its hipGraphExec handles belong to the graphs a re-capture replaces
        self._fast = None
        if self._device_p2p and self._copy_stream is not None:
            return False  # copy-stream refills beside device edges: the step stays eager
        if self._copy_stream is not None or (self.prog.has_comm and not self._device_p2p):
            return self.capture_segments()
        self._sync()
        self._retire_native()
        if self._device_p2p:
            # (on this rank's own stream: a warm step spinning on a peer's flag from a pooled side
            # stream could share a hardware queue with that peer's stream — parallel/loopback.py)
            self._step_body(StepStats())
        else:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._step_body(StepStats())  # warm the residency state on the capture stream
            torch.cuda.current_stream(self.device).wait_stream(s)
        self._sync()
        # captured on a side stream without torch.cuda.graph's device-wide synchronize (ranks
        # sharing one GPU may be capturing their own graphs meanwhile)
        # (kept until this executor dies, then destroyed at a quiesce point: parallel/lifetime.py)
        g = lifetime.keep(self, torch.cuda.CUDAGraph(keep_graph=True))
        cur = torch.cuda.current_stream(self.device)
        if self._cap_stream is None:
            self._cap_stream = torch.cuda.Stream(self.device)
        self._cap_stream.wait_stream(cur)
        with torch.cuda.stream(self._cap_stream):
            g.capture_begin(capture_error_mode="thread_local")
            try:
                self._step_body(StepStats())
            finally:
                g.capture_end()
        cur.wait_stream(self._cap_stream)
        self.launches = ops.ext().graph_kernel_nodes(g.raw_cuda_graph())
        g.instantiate()
        self._sync()
        self._graph = g
        self._graph_exec = g.raw_cuda_graph_exec()
        if not (self.trace or self.debug):
            # step()'s fast path: the launch function, its arguments, the (static) stats
            # (the stream current at capture: the rank's own, where every later step is issued)
            self._fast = (ops.ext().graph_launch, self._graph_exec, cur.cuda_stream,
                          StepStats(kernels=self.prog.n_kernels), self._device_p2p or self._attn_sync is not None)
        return True

    def _sync(self) -> None:
        """Wait for this executor's own streams (compute, copy, capture). Not a device-wide
        synchronize: ranks sharing one GPU (parallel/loopback.py) may be capturing hipGraphs on
        their streams meanwhile, and a device synchronize is illegal during any capture."""
        torch.cuda.current_stream(self.device).synchronize()
        for st in (self._copy_stream, self._cap_stream):
            if st is not None:
                st.synchronize()

    def _retire_native(self) -> None:
        """Before a (re-)capture, after a device synchronize: the graphs / runner of the previous
        capture are replaced — hand them to the graveyard (destroyed at a quiesce point; on the
        main thread right away) instead of keeping every capture alive until the executor dies."""
        self._graph = self._graph_exec = None
        self._segments = {}
        self._drop_runner()
        self._fast = None
        lifetime.retire(self)
        lifetime.release_on_main_thread()

    def _drop_runner(self) -> None:
        self._runner = None
        self._runner_stats = None
        self.issue_mode = None

    def _plan_segments(self) -> List[Tuple[int, int]]:
        """[start, end) ranges of consecutive ``run`` instructions that replay as one hipGraph.
        Everything a run waits for (a copy-stream fill, a peer's parameter group, a received
        activation, an in-flight send of its output region) happens eagerly BEFORE its segment,
        so such a run starts a segment (waiting earlier inside one would delay the runs before
        it); a prefetch issue point (the copy stream waits for the compute stream there) ends
        one. Non-run instructions (loads, evictions, p2p) stay eager between segments."""
        pre = set(sum(self._hoist.values(), [])) | set(sum(self._carry_at.values(), []))
        fresh: set = set()  # groups / activations whose first reader must start a segment
        received = set()
        starts, ends = set(), set()
        for i, ins in enumerate(self.prog.instrs):
            if ins.op == "load" and (i in pre or ins.peer >= 0):
                fresh.add(ins.param)
            elif ins.op == "recv":
                received.add(ins.task)
            elif ins.op == "run":
                needs = set()
                deps = set()
                for tid in ins.group:
                    needs |= self.tasks[tid].params_needed
                    deps |= set(self.tasks[tid].dependencies)
                if needs & fresh or deps & received or ins.wait_sends:
                    starts.add(i)
                fresh -= needs
                received -= deps
                if i in self._hoist or i in self._carry_at:
                    ends.add(i)
        segs: List[Tuple[int, int]] = []
        i, n = 0, len(self.prog.instrs)
        while i < n:
            if self.prog.instrs[i].op != "run":
                i += 1
                continue
            j = i + 1
            while j < n and self.prog.instrs[j].op == "run" and j not in starts and (j - 1) not in ends:
                j += 1
            segs.append((i, j))
            i = j
        return segs

    def _capture_segment(self, i: int, seg_end: int, stats: StepStats):
        """Record runs [i, seg_end) into a hipGraph WITHOUT a device-wide synchronize
        (``torch.cuda.graph`` synchronizes on entry, which would make every eager isend /
        irecv / parameter send posted earlier in this step host-blocking — two ranks exchanging
        in opposite directions could then wait on each other at capture). The capture runs on
        a side stream ordered after the compute stream; the compute stream waits for it."""
        if all(k in self._moe_skip or k in self._mlp_skip or k in self._xskip for k in range(i, seg_end)):
            return None  # its runs issue with a batch elsewhere: no graph at all
        g = lifetime.keep(self, torch.cuda.CUDAGraph(keep_graph=True))
        cur = torch.cuda.current_stream(self.device)
        if self._cap_stream is None:
            self._cap_stream = torch.cuda.Stream(self.device)
        cs = self._cap_stream
        cs.wait_stream(cur)
        with torch.cuda.stream(cs):
            # thread-local capture mode: RCCL's watchdog thread keeps querying its events
            g.capture_begin(pool=self._seg_pool, capture_error_mode="thread_local")
            try:
                for k in range(i, seg_end):
                    self._issue_run(k, self.prog.instrs[k], stats, None)
            except BaseException:
                # an error inside a capture can end in an abort when the graph is torn down,
                # which hides it: report the cause first
                import traceback
                traceback.print_exc()
                raise
            finally:
                g.capture_end()
            self.launches = (self.launches or 0) + ops.ext().graph_kernel_nodes(g.raw_cuda_graph())
            if ops.ext().graph_nodes(g.raw_cuda_graph()) == 0:
                # every run of the segment was folded into another launch (a norm written by its
                # producer, say): nothing to replay — no graph launch per step for it. The empty
                # graph is not destroyed here (lifetime.keep): tearing a graph down while another
                # rank's thread of the single-GPU harness is capturing aborted the process
                cur.wait_stream(cs)
                return None
            g.instantiate()
        cur.wait_stream(cs)
        return g

    def _runner_ok(self) -> bool:
        """Can this rank's steady-state step be recorded for the native runner? Every run is in
        a captured segment and every steady-state refill copies a host image."""
        if not RUNNER or self.trace or self.debug:
            return False
        if not ((self.gpu and self._segments) or (not self.gpu and RUNNER_CPU)):
            return False
        if self._refills() and self.gpu:
            for i in self.prog.instrs:
                if i.op == "load" and i.peer < 0 and self._img_override.get(i.param) is None:
                    img = self.store.group_image(i.param)
                    if img is None or not img.is_pinned():
                        return False
        return True

    def build_runner(self) -> bool:
        """Record one steady-state step (a dry run of the issue loop: every device action goes
        to a native StepRunner instead of the device), then execute it; later steps are one
        ``StepRunner.run()`` each (csrc/kernels/runner.cpp). Host bookkeeping is cyclic in the
        steady state, so the recorded step is every step."""
        if not self._runner_ok():
            return False
        if self.gpu:
            self._sync()  # the previous steps' cross-step fills are complete
        r = lifetime.keep(self, ops.ext().StepRunner())
        if self._copy_stream is not None:
            r.set_copy_stream(self._copy_stream.cuda_stream)
        if self.comm is not None and self.comm.kind == "loopback":
            r.set_loopback(self.comm.hub, self.comm.rank)
        elif self.pg is not None:
            r.set_process_group(self.pg)
        self._rec = _Recorder(r)
        stats = StepStats()
        try:
            self._step_body(stats)
        finally:
            self._rec = None
        r.run()  # ... the recorded step, executed
        self._runner, self._runner_stats = r, stats
        self.issue_mode = "runner"
        return True

    def _leave_runner(self) -> None:
        """Back to the Python issue loop (a profiled step): the runner's cross-step fills become
        plain completed work."""
        if self.gpu:
            self._sync()
        self._runner = None
        self._carry = {}
        self._await = {}
        self.issue_mode = "python"

    def capture_segments(self) -> bool:
        """Piecewise capture for programs that must stay eager around RCCL p2p or copy-stream
        refills: one hipGraph per kernel-group segment (_plan_segments), sharing one memory
        pool, captured in program order during a steady-state step (the host bookkeeping of
        that step runs as usual; its segment kernels are recorded, not run)."""
        self._segments = {}
        self.launches = None
        segs = [(a, b) for a, b in self._plan_segments()]
        if not segs:
            if self.prog.has_comm:  # stay in p2p step with the ranks that capture (two steps below)
                self.step()
                self.step()
            return False
        self._sync()
        self._retire_native()
        self._capture_plan = {a: b for a, b in segs}
        self._seg_pool = torch.cuda.graph_pool_handle()
        self._step_body(StepStats())  # segments captured in order as the step reaches them
        self._capture_plan = None
        self._sync()
        built = bool(self._segments) and self.build_runner()
        if not built and self.prog.has_comm:
            # build_runner executes the step it recorded; a rank that could not record one runs
            # a step from the Python loop instead, so every rank of a p2p program has executed
            # the same number of steps (their transfers pair step by step) whichever path it takes
            self.step()
        if built and RUNNER_MODE == "auto" and not self.prog.has_comm:
            self._pick_issue_mode()
        return bool(self._segments)

    def _pick_issue_mode(self, n: int = 3) -> None:
        """Keep the native runner or the Python issue loop, whichever runs this rank's steps
        faster (comm-free programs only: with p2p a rank's step time also depends on its peers).
        The loop paces the issue of copy-stream fills at host speed, which on copy-bound steps
        can beat issuing the whole step at once."""
        def timed():
            self._sync()
            t0 = time.perf_counter()
            for _ in range(n):
                self.step()
            self._sync()
            return (time.perf_counter() - t0) / n
        t_runner = timed()
        self._leave_runner()
        self.step()  # the loop's first step re-issues the fills the runner carried across steps
        t_loop = timed()
        if t_loop < 0.98 * t_runner:
            self.issue_mode = "python"
            return
        self.build_runner()
        self.issue_mode = "runner"

    def refine_tuning(self, top: int = 3, reps: int = 20, min_gain: float = 0.01, force: bool = False,
                      exhaustive: bool = False, log=None, cfgs=None, keys=None) -> Dict:
        """GEMM config choice by WHOLE-STEP time: for every GEMM shape this rank runs (costliest
        first), try the microbenchmark's runner-up configs inside the captured hipGraph of the
        real step and keep one only if the step gets faster by > ``min_gain``. The cold-weight
        microbenchmark misses the DAG's cache state and neighbour kernels; this does not.
        ``exhaustive``: every valid (config, split-K <= 4) of the shape instead of the runner-ups
        (``log(key, cand, ms)`` sees each timing); ``cfgs``: only candidates with these config ids
        (e.g. newly added tile configs against the current choice); ``keys``: only these shape
        keys ("MxNxK[tag]"). Persists the choices (ops/gemm_tuning.json).
        Returns {key: (old, new, step_ms)}."""
        from ..ops import tuning

        if not (self.gpu and self.use_graph) or self._copy_stream is not None or self.prog.has_comm:
            return {}  # whole-step graphs only

        def step_ms():
            self._graph = self._graph_exec = self._fast = None
            self.capture()
            for _ in range(3):
                self._graph.replay()
            torch.cuda.synchronize(self.device)
            ts = []
            for _ in range(3):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(reps):
                    self._graph.replay()
                b.record()
                torch.cuda.synchronize(self.device)
                ts.append(a.elapsed_time(b) / reps)
            return sorted(ts)[1]

        shapes = sorted(self.gemm_shapes(), key=lambda s: -(s[0] * s[1] * s[2]))
        if keys:
            shapes = [s for s in shapes if f"{s[0]}x{s[1]}x{s[2]}{s[3]}" in keys]
        base = step_ms()
        if log is not None:
            log("baseline", (), base)
        changes = {}
        for sh in shapes:
            M, N, K, tg = sh
            if tuning.is_refined(M, N, K, tg) and not force:
                continue
            if not tuning.runner_ups(M, N, K, tg):  # no microbenchmark ranking kept: make one
                prev = tuning.table().get(tuning._key(M, N, K, tg))
                tuning.tune(M, N, K, device=self.device, save=False, tg=tg)
                if prev is not None:
                    tuning.set_choice(M, N, K, tg, prev)
            cur = tuning.lookup(M, N, K, tg)
            best, best_ms = cur, base
            if exhaustive:
                cands = [c for c in tuning.candidates(M, N, K, ops.ext().gemm_glds_num_configs(), tg)
                         if c[1] <= 4 and (c[0] < tuning.REGSTAGE or c[0] == tuning.LIB)]
            else:
                cands = tuning.runner_ups(M, N, K, tg, top + 1)
            if cfgs:
                cands = [c for c in tuning.candidates(M, N, K, ops.ext().gemm_glds_num_configs(), tg)
                         if c[0] in cfgs and c[1] <= 4]
            for cand in cands:
                if tuple(cand) == tuple(cur):
                    continue
                tuning.set_choice(M, N, K, tg, cand)
                try:
                    ms = step_ms()
                except RuntimeError:  # a config this shape / epilogue cannot run
                    continue
                if log is not None:
                    log(f"{M}x{N}x{K}{tg}", tuple(cand), ms)
                if ms < best_ms * (1.0 - min_gain):
                    best, best_ms = tuple(cand), ms
            tuning.set_choice(M, N, K, tg, best)
            tuning.mark_refined(M, N, K, tg)
            if tuple(best) != tuple(cur):
                changes[f"{M}x{N}x{K}{tg}"] = (tuple(cur), tuple(best), round(best_ms, 4))
                base = best_ms
        tuning.save()
        self._graph = self._graph_exec = self._fast = None
        self.capture()
        return changes

    def output(self, tid: str) -> torch.Tensor:
        """The output of task ``tid``; for a request merged into a micro-batch group
        (runtime.plan merge_mb), its batch rows of the merged task's output."""
        if tid in self._views or "/" not in tid:
            return self._views[tid]
        rid, base = tid.split("/", 1)
        merged, lo, hi = self.requests[rid + "/"]
        return self._views[merged + base][lo:hi]

    def owns_output(self, tid: str) -> bool:
        """Does this rank hold ``tid``'s output (merged requests resolved)?"""
        if tid in self._views:
            return True
        if "/" in tid:
            rid, base = tid.split("/", 1)
            m = self.requests.get(rid + "/")
            return m is not None and (m[0] + base) in self._views
        return False

    def memory_bytes(self) -> Dict[str, int]:
        return {"activations": self.act_slab.numel(), "params": self.param_slab.numel(),
                "workspace": self.ws_slab.numel()}
