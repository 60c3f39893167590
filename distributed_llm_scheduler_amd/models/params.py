"""Parameter groups: scheduler parameter ids -> the real tensors behind them.

The scheduler reasons about opaque parameter ids (``"layer_3_attn_qkv_weights"``); the
executor needs bytes. A :class:`ParamGroup` lists the tensors one id stands for, in the
layout the HIP kernels consume:

* every GEMM weight is stored **[N][K] (K contiguous)**, bf16, so both MFMA operands of
  ``y = x @ W^T`` stream K-contiguous rows (GPT-2's Conv1D stores [K][N]; the checkpoint
  converter transposes once at load time, never per call);
* norms/biases are bf16 vectors (the kernels accumulate in fp32).

Initialisation is deterministic per tensor name (random-init weights of the named
architecture; there are no checkpoints offline).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch


@dataclass
class TensorSpec:
    name: str
    shape: Tuple[int, ...]
    init: str = "normal"  # normal | ln | bias | ones | zeros
    std: float = 0.02
    parent: Optional["TensorSpec"] = None  # shard of a larger tensor (tensor parallelism)
    slc: Optional[tuple] = None            # (dim, start, stop) or ("rows", ((a, b), ...))

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclass
class ParamGroup:
    pid: str
    tensors: List[TensorSpec] = field(default_factory=list)

    def nbytes(self, dtype_bytes: int = 2) -> int:
        return sum(t.numel for t in self.tensors) * dtype_bytes


def _seed(name: str, base: int) -> int:
    return (int(hashlib.sha1(name.encode()).hexdigest()[:12], 16) + base) % (2 ** 62)


def _take(full: torch.Tensor, slc) -> torch.Tensor:
    if slc[0] == "rows":
        return torch.cat([full[a:b] for a, b in slc[1]], 0).contiguous()
    dim, a, b = slc
    return full.narrow(dim, a, b - a).contiguous()


def materialize(spec: TensorSpec, dtype=torch.bfloat16, device="cpu", seed: int = 0) -> torch.Tensor:
    """Deterministic random-init tensor for ``spec`` (fp32 generation, cast once). A shard
    is the matching slice of its parent, so sharded and unsharded models are identical."""
    if spec.parent is not None:
        return _take(materialize(spec.parent, dtype, device, seed), spec.slc)
    if spec.init == "ones":
        return torch.ones(spec.shape, dtype=dtype, device=device)
    if spec.init == "zeros":
        return torch.zeros(spec.shape, dtype=dtype, device=device)
    g = torch.Generator().manual_seed(_seed(spec.name, seed))
    if spec.init == "ln":  # non-trivial LayerNorm/RMSNorm gains so tests exercise them
        t = 1.0 + 0.1 * torch.randn(spec.shape, generator=g)
    elif spec.init == "bias":
        t = 0.02 * torch.randn(spec.shape, generator=g)
    else:
        t = spec.std * torch.randn(spec.shape, generator=g)
    return t.to(dtype=dtype, device=device)


def fill_on_device(spec: TensorSpec, out: torch.Tensor, seed: int = 0) -> None:
    """Random-init ``out`` (already in HBM) for ``spec`` with the device RNG: no host
    master copy, no PCIe traffic — how the large-model benchmarks (Llama-3-8B 16 GB,
    Mixtral-8x7B 93 GB) get their weights. Deterministic per name, but a different
    stream from :func:`materialize` (so not comparable to the CPU reference)."""
    if spec.parent is not None:
        full = torch.empty(spec.parent.shape, dtype=out.dtype, device=out.device)
        fill_on_device(spec.parent, full, seed)
        out.copy_(_take(full, spec.slc))
        return
    if spec.init == "ones":
        out.fill_(1.0)
        return
    if spec.init == "zeros":
        out.zero_()
        return
    g = torch.Generator(device=out.device).manual_seed(_seed(spec.name, seed))
    if spec.init == "ln":
        out.normal_(1.0, 0.1, generator=g)
    elif spec.init == "bias":
        out.normal_(0.0, 0.02, generator=g)
    else:
        out.normal_(0.0, spec.std, generator=g)


class ParamStore:
    """Host-side master copy of every parameter group (pinned when a GPU is present),
    materialised lazily; the executor copies groups into its HBM arena on demand.
    ``device_init=True`` skips the host copy: groups are random-initialised directly in
    the arena (benchmarks of models whose host materialisation would dominate setup)."""

    def __init__(self, groups: Dict[str, ParamGroup], dtype=torch.bfloat16, seed: int = 0, pin: bool = None,
                 device_init: bool = False):
        self.groups = groups
        self.dtype = dtype
        self.seed = seed
        self.device_init = device_init
        self.pin = (torch.cuda.is_available() and not device_init) if pin is None else pin
        self._host: Dict[str, torch.Tensor] = {}
        self._images: Dict[str, torch.Tensor] = {}
        self._specs: Dict[str, TensorSpec] = {}
        for g in groups.values():
            for sp in g.tensors:
                while sp is not None:  # shards and the full tensors they slice
                    self._specs.setdefault(sp.name, sp)
                    sp = sp.parent

    def tensor(self, name: str) -> torch.Tensor:
        t = self._host.get(name)
        if t is None:
            spec = self._spec(name)
            if spec.parent is not None:
                t = _take(self.tensor(spec.parent.name), spec.slc)
            else:
                t = materialize(spec, self.dtype, "cpu", self.seed)
            if self.pin:
                t = t.pin_memory()
            self._host[name] = t
        return t

    def _spec(self, name: str) -> TensorSpec:
        return self._specs[name]

    def fill(self, name: str, out: torch.Tensor) -> None:
        """Write tensor ``name`` into ``out`` (an HBM arena view)."""
        if self.device_init and out.is_cuda and name not in self._host:
            fill_on_device(self._spec(name), out, self.seed)
        else:
            out.copy_(self.tensor(name), non_blocking=True)

    def group_image(self, pid: str) -> Optional[torch.Tensor]:
        """The group as ONE host byte image in its arena layout (pinned), so a refill is a
        single DMA of the whole group instead of a copy per tensor; ``None`` for
        device-initialised stores (nothing on the host to copy)."""
        if self.device_init:
            return None
        img = self._images.get(pid)
        if img is None:
            total, layout = group_layout(self.groups[pid], torch.tensor([], dtype=self.dtype).element_size())
            img = torch.zeros(total, dtype=torch.uint8)
            for spec, off in layout:
                t = self.tensor(spec.name).contiguous()
                img[off:off + t.numel() * t.element_size()].copy_(t.view(-1).view(torch.uint8))
            if self.pin:
                img = img.pin_memory()
            self._images[pid] = img
        return img

    def group_tensors(self, pid: str) -> List[Tuple[TensorSpec, torch.Tensor]]:
        return [(s, self.tensor(s.name)) for s in self.groups[pid].tensors]

    def nbytes(self, pid: str) -> int:
        """Bytes the group occupies in the HBM parameter arena (256-B aligned tensors)."""
        return group_layout(self.groups[pid], torch.tensor([], dtype=self.dtype).element_size())[0]

    def set_tensor(self, name: str, value: torch.Tensor) -> None:
        """Install real weights (e.g. converted from a checkpoint) for ``name``."""
        spec = self._spec(name)
        if tuple(value.shape) != tuple(spec.shape):
            raise ValueError(f"{name}: expected shape {spec.shape}, got {tuple(value.shape)}")
        t = value.detach().to("cpu", self.dtype).contiguous()
        self._host[name] = t.pin_memory() if self.pin else t
        self._images = {k: v for k, v in self._images.items()
                        if all(sp.name != name for sp in self.groups[k].tensors)}


GROUP_ALIGN = 256


def group_layout(group: ParamGroup, dtype_bytes: int = 2):
    """Byte layout of a parameter group inside the HBM parameter arena: every tensor
    starts 256-B aligned (16-B vector loads, cache-line aligned rows).
    Returns ``(total_bytes, [(spec, byte_offset), ...])``."""
    off, out = 0, []
    for spec in group.tensors:
        out.append((spec, off))
        off += (spec.numel * dtype_bytes + GROUP_ALIGN - 1) // GROUP_ALIGN * GROUP_ALIGN
    return off, out
