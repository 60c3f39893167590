"""GEMM autotuning for MI355X.

Every distinct (M, N, K) the executor will run is timed over the LDS-DMA kernel's tile
configs x split-K factors (plus the register-staged kernel) and the fastest choice is
cached — in memory, and in ``gemm_tuning.json`` next to this file so tuned shapes ship with
the repository. Measurement regime matches the DAG's: weights are COLD (a ring of weight
copies larger than the 256 MiB Infinity Cache is rotated, so each call streams its weights
from HBM as a once-per-step layer does), launches are captured in a hipGraph so host launch
cost does not hide device time, and the median of several rounds is kept.
"""
from __future__ import annotations

import json
import os
import statistics
import threading
from typing import Dict, Iterable, Optional, Tuple

import torch

_PATH = os.environ.get("DLS_GEMM_TUNING") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "gemm_tuning.json")
_lock = threading.Lock()
_table: Optional[Dict[str, Tuple[int, int]]] = None
_cands: Dict[str, list] = {}     # key -> runner-up (cfg, splitk) by microbenchmark time (for in-DAG refinement)
_refined: Dict[str, bool] = {}   # key -> chosen by whole-step timing inside a DAG
# key -> [(first column, end column, config, splitk), ...]: the GEMM runs as one launch per
# column range (a wide GEMM whose tile count is 1.5 rounds of the 256 CUs: a whole round of big
# tiles, then the remaining columns as ONE round of narrower tiles)
_col_splits: Dict[str, list] = {}
# model -> {key: choice}: a model whose step measured faster with another config for a shape it
# shares with other models (Mixtral-8x7B's QKV GEMM after the MoE layer vs Llama-3-8B's)
_overrides: Dict[str, Dict[str, Tuple[int, int]]] = {}
_model: Optional[str] = None
REGSTAGE = 100  # config ids >= 100 select the register-staged kernel (csrc ops_binding kRegStage)
PERSIST = 64    # config | 64: the same LDS-DMA tile config as a persistent launch (kernels.h kGemmPersist)
LIB = 200       # the vendor library (hipBLASLt through torch.mm): OFF unless DLS_ALLOW_VENDOR_GEMM=1
                # (then a candidate for PLAIN GEMMs only — a GEMM with a fused epilogue always
                # runs on the HIP kernels). Default: every GEMM runs on the hand-written kernels,
                # and a table entry naming LIB resolves to the best HIP candidate (lookup)
VENDOR = os.environ.get("DLS_ALLOW_VENDOR_GEMM", "0") == "1"


def _key(M: int, N: int, K: int, tg: str = "") -> str:
    return f"{M}x{N}x{K}{tg}"


def tag(act: int = 0, ranged: bool = False) -> str:
    """Variant suffix of a tuning key: SwiGLU epilogue ("s"), device row range ("r")."""
    return ("s" if act == 4 else "") + ("r" if ranged else "")


def table() -> Dict[str, Tuple[int, int]]:
    global _table
    with _lock:
        if _table is None:
            _table = {}
            if os.path.exists(_PATH):
                try:
                    with open(_PATH) as f:
                        doc = json.load(f)
                    _table = {k: tuple(v) for k, v in doc.get("gemm", {}).items()}
                    _cands.update({k: [tuple(c) for c in v] for k, v in doc.get("candidates", {}).items()})
                    _refined.update(doc.get("refined", {}))
                    _col_splits.update({k: [tuple(x) for x in v] for k, v in doc.get("col_splits", {}).items()})
                    _overrides.update({m: {k: tuple(v) for k, v in t.items()}
                                       for m, t in doc.get("model_overrides", {}).items()})
                except (OSError, ValueError):
                    _table = {}
        return _table


def set_model(name: Optional[str]) -> None:
    """The model whose step the following GEMMs belong to (its ``model_overrides`` apply)."""
    global _model
    _model = name


def lookup(M: int, N: int, K: int, tg: str = "") -> Tuple[int, int]:
    """(config, splitk) for this shape/variant: the current model's override if it has one,
    else tuned if known (a variant falls back to the plain shape's LDS-DMA choice), else
    (-1, 0) = kernel heuristic."""
    t = table()
    v = _overrides.get(_model, {}).get(_key(M, N, K, tg))
    if v is not None:
        return v
    v = t.get(_key(M, N, K, tg))
    if v is None and tg:
        v = t.get(_key(M, N, K))
        if v is not None and v[0] >= REGSTAGE:
            v = None
    if v is not None and v[0] == LIB and not VENDOR:
        v = _hip_candidate(M, N, K, tg)
    return v if v is not None else (-1, 0)


def _hip_candidate(M: int, N: int, K: int, tg: str = ""):
    """The fastest hand-written-kernel candidate of the shape's microbenchmark, else None."""
    for c in _cands.get(_key(M, N, K, tg), []):
        if c[0] != LIB:
            return tuple(c)
    return None


def col_split(M: int, N: int, K: int, tg: str = ""):
    """[(n0, n1, config, splitk), ...] if (M, N, K[, variant]) runs as several column-range
    launches (``col_splits`` of the table; ``DLS_COL_SPLIT=0`` disables), else None."""
    if os.environ.get("DLS_COL_SPLIT", "1") == "0":
        return None
    table()
    return _col_splits.get(_key(M, N, K, tg))


def lookup_fused(M: int, N: int, K: int, tg: str = "") -> Tuple[int, int]:
    """Like :func:`lookup`, for a GEMM with a fused epilogue (which the vendor library cannot
    run): if the tuned choice is ``LIB``, the fastest HIP-kernel candidate of the same
    microbenchmark instead of the kernel's heuristic."""
    cfg, sk = lookup(M, N, K, tg)
    if cfg != LIB:
        return cfg, sk
    return _hip_candidate(M, N, K, tg) or (-1, 0)


def _save() -> None:
    """Write the table atomically (temp file + rename): the ranks of a multi-GPU job share the
    file, and a reader must never see a half-written one."""
    tmp = f"{_PATH}.{os.getpid()}.tmp"
    try:
        with open(tmp, "w") as f:
            json.dump({"device": "MI355X (gfx950)", "gemm": {k: list(v) for k, v in sorted(table().items())},
                       "candidates": {k: [list(c) for c in v] for k, v in sorted(_cands.items())},
                       "refined": dict(sorted(_refined.items())),
                       "col_splits": {k: [list(x) for x in v] for k, v in sorted(_col_splits.items())},
                       "model_overrides": {m: {k: list(v) for k, v in sorted(t.items())}
                                           for m, t in sorted(_overrides.items())}}, f, indent=1)
        os.replace(tmp, _PATH)
    except OSError:
        try:
            os.remove(tmp)
        except OSError:
            pass


def _graph_time(fn, reps: int = 10, rounds: int = 5) -> float:
    """Median device time (us) of ``fn`` per call, measured on a hipGraph of ``reps`` calls."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(res)


# csrc gemm_glds kKStep: K granularity per LDS-DMA config id (64; 128 / 256 for two / four K groups)
_KSTEP = [64] * 16 + [128] * 4 + [256] * 2 + [64] * 3 + [128] * 4 + [64, 128, 64, 64, 64] + [64, 64] + [64, 64, 64, 128, 128, 64] + [64] + [64] + [64] + [256] + [64, 64]
# configs whose 48- / 112- / 144-column wave tiles cannot pair SwiGLU gate/up fragments
SWIGLU_BAD = frozenset(range(22, 28)) | {36, 38, 39, 42, 45}


def kstep(cfg: int) -> int:
    """K granularity of an LDS-DMA config (csrc gemm_glds kKStep)."""
    c = cfg % PERSIST if cfg < REGSTAGE else 0
    return _KSTEP[c] if c < len(_KSTEP) else 64


def candidates(M: int, N: int, K: int, n_cfg: int, tg: str = ""):
    out = [] if tg else [(REGSTAGE + 0, 1), (REGSTAGE + 2, 1), (REGSTAGE + 3, 1)] + ([(LIB, 1)] if VENDOR else [])
    for cfg in range(n_cfg):
        ks = kstep(cfg)
        if cfg in SWIGLU_BAD and "s" in tg:
            continue  # 48/144-column wave tiles cannot pair SwiGLU gate/up fragments
        for sk in ((1,) if "g" in tg else (1, 2, 3, 4, 6, 8)):  # grouped launches: no split-K
            if K % 64 or K % (ks * sk) or (sk > 1 and N % 8) or K // (ks * sk) < 2:
                continue
            if sk > 1 and M * N > 2048 * 8192:
                continue
            out.append((cfg, sk))
    if M * N >= (8 << 20) and K % 64 == 0 and not tg:
        # many more tiles than resident blocks (LM heads): the persistent tile walk of the
        # 256x128 / 64x64 configs (kernels.h kGemmPersist = 64)
        out += [(PERSIST + c, 1) for c in (0, 3, 14) if c < n_cfg]
    return out


def tune(M: int, N: int, K: int, device=None, cold: bool = True, save: bool = True, verbose: bool = False,
         tg: str = ""):
    """Time every candidate for (M, N, K[, variant]) and record the fastest. Returns
    ((cfg, splitk, us), {candidate: us}). A ranged variant ("r") is timed as an M-row range
    inside a grid sized for 4 M rows (how MoE experts launch)."""
    from . import ext

    e = ext()
    dev = device or torch.device("cuda")
    act = 4 if "s" in tg else 0
    if "g" in tg:
        return _tune_grouped(e, M, N, K, dev, act, tg, save)
    rows_total = 4 * M if "r" in tg else M
    x = (torch.randn(rows_total, K, device=dev) * 0.5).bfloat16()
    rng = torch.tensor([M, 2 * M], dtype=torch.int32, device=dev) if "r" in tg else None
    wbytes = N * K * 2
    copies = max(1, min(64, (512 << 20) // max(wbytes, 1) + 1)) if cold else 1
    ws = [(torch.randn(N, K, device=dev) * 0.05).bfloat16() for _ in range(copies)]
    out = torch.empty(rows_total, N // 2 if act == 4 else N, device=dev, dtype=torch.bfloat16)
    best = None
    results = {}
    for cfg, sk in candidates(M, N, K, e.gemm_glds_num_configs(), tg):
        try:
            if cfg == LIB:
                t = _graph_time(lambda i: torch.mm(x, ws[i % copies].t(), out=out))
            else:
                t = _graph_time(lambda i: e.gemm(x, ws[i % copies], None, None, act, 1.0, out, cfg, sk, None, 0,
                                                 1e-5, rng))
        except RuntimeError:
            continue
        results[(cfg, sk)] = t
        if best is None or t < best[2]:
            best = (cfg, sk, t)
        if verbose:
            print(f"  {M}x{N}x{K} cfg={cfg} splitk={sk}: {t:.2f} us")
    del ws
    if best is not None:
        table()[_key(M, N, K, tg)] = (best[0], best[1])
        _cands[_key(M, N, K, tg)] = [c for c, _ in sorted(results.items(), key=lambda kv: kv[1])[:4]]
        if save:
            _save()
    return best, results


GROUPS = 8  # experts per grouped microbenchmark launch (Mixtral-8x7B)


def _tune_grouped(e, M: int, N: int, K: int, dev, act: int, tg: str, save: bool):
    """Grouped MoE-expert launch ("g" variants): GROUPS experts of M routed rows each, every
    expert its own weight (together far beyond the Infinity Cache: cold by construction)."""
    E = GROUPS
    x = (torch.randn(E * M, K, device=dev) * 0.5).bfloat16()
    ws = [(torch.randn(N, K, device=dev) * 0.05).bfloat16() for _ in range(E)]
    wp = torch.tensor([w.data_ptr() for w in ws], dtype=torch.int64, device=dev)
    # routed-row counts as top-k routing of random tokens spreads them (multinomial around M,
    # so about half the experts get MORE than M rows — what a tile height must absorb)
    g = torch.Generator().manual_seed(7)
    cnt = torch.bincount(torch.randint(0, E, (E * M,), generator=g), minlength=E)
    off = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)]).to(torch.int32).to(dev)
    if act == 4:
        out, outs, op = torch.empty(E * M, N // 2, device=dev, dtype=torch.bfloat16), [], None
    else:
        out = None
        outs = [torch.empty(2 * M, N, device=dev, dtype=torch.bfloat16) for _ in range(E)]
        op = torch.tensor([o.data_ptr() for o in outs], dtype=torch.int64, device=dev)
    best, results = None, {}
    for cfg, sk in candidates(M, N, K, e.gemm_glds_num_configs(), tg):
        try:
            t = _graph_time(lambda i: e.gemm_grouped(x, ws, wp, off, act, out, outs, op, cfg), reps=4)
        except RuntimeError:
            continue
        results[(cfg, sk)] = t
        if best is None or t < best[2]:
            best = (cfg, sk, t)
    del ws
    if best is not None:
        table()[_key(M, N, K, tg)] = (best[0], best[1])
        _cands[_key(M, N, K, tg)] = [c for c, _ in sorted(results.items(), key=lambda kv: kv[1])[:4]]
        if save:
            _save()
    return best, results


def set_choice(M: int, N: int, K: int, tg: str, choice: Tuple[int, int]) -> None:
    k = _key(M, N, K, tg)
    if k in _overrides.get(_model, {}):  # the current model's own choice for a shared shape
        _overrides[_model][k] = tuple(choice)
    else:
        table()[k] = tuple(choice)


def runner_ups(M: int, N: int, K: int, tg: str = "", n: int = 3) -> list:
    return [c for c in _cands.get(_key(M, N, K, tg), []) if VENDOR or c[0] != LIB][:n]


def mark_refined(M: int, N: int, K: int, tg: str = "") -> None:
    _refined[_key(M, N, K, tg)] = True


def is_refined(M: int, N: int, K: int, tg: str = "") -> bool:
    return bool(_refined.get(_key(M, N, K, tg)))


def save() -> None:
    _save()


def ensure_tuned(shapes: Iterable[tuple], device=None) -> None:
    """Tune every (M, N, K[, variant]) not yet in the table (called by the executor at setup)."""
    tuned = False
    for sh in sorted(set(shapes)):
        M, N, K = sh[:3]
        tg = sh[3] if len(sh) > 3 else ""
        if _key(M, N, K, tg) not in table():
            tune(M, N, K, device=device, save=False, tg=tg)
            tuned = True
    if tuned:  # every shape already known (the usual case, all ranks): leave the file alone
        _save()
