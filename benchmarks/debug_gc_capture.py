"""Debug: the lifetime GPU test's steps with flushed progress prints (finds a silent exit)."""
import gc
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_scheduler_amd.parallel import lifetime, runtime  # noqa: E402


def say(*a):
    print(*a, flush=True)


mode = sys.argv[1] if len(sys.argv) > 1 else "all"
dev = torch.device("cuda:0")
say("plan")
p = runtime.plan("mini-gpt2", world=1, seq=64)
ex = runtime.make_executor(p, 0, dev, runtime.make_store(p), use_graph=True)
say("step")
ex.step()
say("capture", ex.capture())
ex.step()
torch.cuda.synchronize()
say("captured step ok; keep", len(ex.__dict__.get("_native_keep", [])))
ex._cycle = ex
del ex
if mode == "nogc":
    say("skip gc")
inside, collected, err = threading.Event(), threading.Event(), []
x = torch.randn(256, 256, device=dev)
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream(dev)
out = {}


def capture():
    try:
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            say("T: capture_begin")
            g.capture_begin(capture_error_mode="thread_local")
            try:
                y = x @ x if mode != "relu" else x * 2
                say("T: inside")
                inside.set()
                assert collected.wait(60)
                out["o"] = torch.relu(y) + 1
                say("T: ops after gc issued")
            finally:
                g.capture_end()
                say("T: capture_end")
    except BaseException as e:  # noqa: BLE001
        say("T: error", repr(e))
        err.append(e)
        inside.set()


t = threading.Thread(target=capture)
t.start()
inside.wait(60)
if mode != "nogc":
    say("main: gc.collect")
    gc.collect()
    say("main: collected; graveyard", lifetime.graveyard_size())
collected.set()
t.join(60)
say("joined", err)
g.replay()
torch.cuda.synchronize()
say("replayed", torch.allclose(out["o"], torch.relu(x @ x) + 1, rtol=1e-3, atol=1e-2))
say("released", lifetime.release())
torch.cuda.synchronize()
say("done")
