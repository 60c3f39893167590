"""Phase stamps of the one-launch attention block (attn_block.hip) at GPT-2's shape, and its
event time against the three launches it replaces (QKV GEMM, attention, out-proj)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_scheduler_amd import ops  # noqa: E402

DEV = torch.device("cuda:0")
B, S, H, nh = 1, 512, 768, 12
M = B * S


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (scale * torch.randn(*shape, generator=g)).to(torch.bfloat16).to(DEV)


x = rnd(M, H, scale=2.0, seed=1)
w1, b1 = rnd(3 * H, H, scale=0.04, seed=2), rnd(3 * H, scale=0.1, seed=3)
wo, bo = rnd(H, H, scale=0.03, seed=4), rnd(H, scale=0.1, seed=5)
nw, nb = (1 + 0.2 * rnd(H, seed=6).float()).bfloat16(), rnd(H, scale=0.1, seed=7)
res = rnd(M, H, seed=8)
xf = x.float()
st = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).contiguous()
wd, cs, bd = ops.derive_norm_gemm(w1, nw, nb, b1)
qkv = torch.empty(M, 3 * H, device=DEV, dtype=torch.bfloat16)
o = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
out = torch.empty(M, H, device=DEV, dtype=torch.bfloat16)
so = torch.zeros(M, 2, device=DEV)
sync = ops.attn_block_sync(M, S, B, nh, DEV)
e = ops.ext()


def fused(stamps=None):
    e.attn_block(x, wd, bd, cs, st, 1, 1e-5, qkv, o, wo, bo, res, out, so, B, S, nh, 0.125, sync, 1 << 22, stamps)


def three():
    ops.linear_norm(x, wd, cs, bd, "layernorm", out=qkv, ext_stats=st)
    ops.attention(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], B, S, nh, nh, 64, causal=True, out=o)
    ops.linear(o, wo, bo, residual=res, out=out, stats_out=so)


def graph_us(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    res_ = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        res_.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(res_)


for r in range(3):
    print(f"round {r}: three launches {graph_us(three):.2f} us   one launch {graph_us(fused):.2f} us")
n1, n2, n3 = (M // 64) * 36, (S // 64) * nh * B, (M // 64) * (H // 64)
stamps = torch.zeros(n1 + n2 + n3, 4, dtype=torch.int64, device=DEV)
for _ in range(3):
    fused()
torch.cuda.synchronize()
fused(stamps)
torch.cuda.synchronize()
s_ = stamps.cpu()
t0 = s_[:, 1].min().item()
us = lambda v: v / 100.0  # noqa: E731  (100 MHz)
print(f"first start -> last end {us(s_[:, 3].max().item() - t0):.2f} us, {len(s_)} workgroups; err word {int(sync[-1])}")
for name, lo, hi in (("qkv", 0, n1), ("attention", n1, n1 + n2), ("out-proj", n1 + n2, n1 + n2 + n3)):
    sel = s_[(s_[:, 0] >= lo) & (s_[:, 0] < hi)]
    start = (sel[:, 1] - t0).float() / 100
    wait = (sel[:, 2] - sel[:, 1]).float() / 100
    body = (sel[:, 3] - sel[:, 2]).float() / 100
    end = (sel[:, 3] - t0).float() / 100
    f = lambda t: f"min {t.min():6.2f} med {t.median():6.2f} max {t.max():6.2f}"  # noqa: E731
    print(f"{name:10s} n={len(sel):4d}  start {f(start)} | wait {f(wait)} | body {f(body)} | end {f(end)}")
