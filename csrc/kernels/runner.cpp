// Native step runner: the per-rank issue loop of a steady-state step in C++.
//
// The Python executor (parallel/executor.py) decides WHAT a step does — which kernel-group
// segments (captured hipGraphs) run, which parameter groups are re-filled and on which stream,
// where the copy stream and the compute stream wait for each other, which RCCL p2p sends and
// receives are posted and where each is waited for. A steady-state step does exactly the same
// thing every time, so the executor records that action sequence once (``StepRunner.add_*``
// while it runs one step eagerly) and every later step replays it here with one Python call:
// no interpreter work per instruction (SURVEY §2.3 "C++ runtime", replacing the reference's
// assign = execute loop, /root/reference/schedulers.py:78-104).
//
// Actions: launch a hipGraphExec; pull a pinned host image into HBM with the host-pull kernel;
// hipMemcpyAsync; hipMemsetAsync; record / wait a runner-owned hipEvent on the compute or the
// copy stream; post a p2p send / recv through the c10d ProcessGroup of the Python world (RCCL
// on ROCm, gloo on the CPU test backend — the same ops ``dist.isend`` / ``dist.irecv`` call);
// wait a posted p2p op (stream-side for RCCL); open / close a p2p GROUP (the ops posted between
// are one ncclGroupStart/End through c10d coalescing where the backend supports it, and share
// one work). Every op still outstanding at the end of the step is waited for, as the Python
// step does. ``set_loopback`` routes the p2p actions through the single-GPU loopback hub
// (loopback.hpp) instead of a ProcessGroup: several ranks in one process, one GPU. The action
// loop itself is dls::run_actions (csrc/runtime/p2p_match.h), which the native selftest also
// runs under ASan / TSan against a CPU backend.
#include <torch/extension.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/utils/pybind.h>
#include <c10/hip/HIPStream.h>

#include <string>
#include <vector>

#include "kernels.h"
#include "loopback.hpp"

namespace {

using Action = dls::StepAction<at::Tensor, py::object>;
using dls::ActKind;

// a posted p2p op: a c10d work (RCCL / gloo) or a loopback hub op
struct RunnerWork {
  c10::intrusive_ptr<c10d::Work> w;
  int64_t hub = -1;
  explicit operator bool() const { return (bool)w || hub >= 0; }
};

// the runner's device / transport side of dls::run_actions (csrc/runtime/p2p_match.h)
struct Backend {
  using Work = RunnerWork;
  hipStream_t cs = nullptr, copy = nullptr;
  c10d::ProcessGroup* pg = nullptr;
  LoopbackHub* hub = nullptr;
  int64_t hub_rank = 0;
  c10::DeviceType dev_type = c10::DeviceType::CPU;
  const std::vector<hipEvent_t>* events = nullptr;

  hipStream_t on(const Action& a) const { return a.stream == 1 && copy ? copy : cs; }
  void graph(const Action& a) { C10_HIP_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(a.exec), cs)); }
  void pull(const Action& a) { launch_host_pull(a.src, a.dst, (int64_t)a.bytes, a.blocks, on(a)); }
  void memcpy(const Action& a) { C10_HIP_CHECK(hipMemcpyAsync(a.dst, a.src, a.bytes, hipMemcpyDefault, on(a))); }
  void memset(const Action& a) { C10_HIP_CHECK(hipMemsetAsync(a.dst, a.value, a.bytes, on(a))); }
  void record(const Action& a) { C10_HIP_CHECK(hipEventRecord((*events)[a.index], on(a))); }
  void wait_event(const Action& a) { C10_HIP_CHECK(hipStreamWaitEvent(on(a), (*events)[a.index], 0)); }
  void pycall(const Action& a) {
    py::gil_scoped_acquire g;
    a.fn();
  }
  Work post(const Action& a) {
    Work w;
    if (hub) {
      w.hub = hub->post(a.kind == dls::SEND, a.tensor, hub_rank, a.index);
      return w;
    }
    TORCH_CHECK(pg, "p2p action without a process group");
    std::vector<at::Tensor> ts{a.tensor};
    w.w = a.kind == dls::SEND ? pg->send(ts, a.index, 0) : pg->recv(ts, a.index, 0);
    return w;
  }
  bool group_begin() {
    const bool co = !hub && pg && pg->getBackend(dev_type)->supportsCoalescing();
    if (co) pg->startCoalescing(dev_type);
    return co;
  }
  Work group_end() {
    Work w;
    w.w = pg->endCoalescing(dev_type);
    return w;
  }
  void wait(Work& w) {
    if (w.hub >= 0) hub->wait(w.hub);  // the current stream waits for the hub's copy
    else w.w->wait();                  // RCCL: the current stream waits; gloo: blocks
  }
};

class StepRunner {
 public:
  StepRunner() = default;
  ~StepRunner() {
    for (auto e : events_)
      if (e) (void)hipEventDestroy(e);
  }

  void set_process_group(py::object pg) {
    pg_ = pg.is_none() ? c10::intrusive_ptr<c10d::ProcessGroup>() : pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
  }
  void set_copy_stream(uint64_t s) { copy_ = reinterpret_cast<hipStream_t>(s); }
  void set_loopback(std::shared_ptr<LoopbackHub> hub, int64_t rank) {
    hub_ = std::move(hub);
    hub_rank_ = rank;
  }

  void add_graph(uint64_t exec) {
    TORCH_CHECK(exec != 0, "null hipGraphExec");
    any_device_ = true;
    Action a{dls::GRAPH};
    a.exec = exec;
    acts_.push_back(a);
  }
  void add_pull(const at::Tensor& dst, const at::Tensor& src, int64_t bytes, int64_t blocks, int64_t stream) {
    TORCH_CHECK(dst.is_cuda() && src.is_pinned(), "pull: device destination, pinned host source");
    TORCH_CHECK(dst.nbytes() >= (size_t)bytes && src.nbytes() >= (size_t)bytes && bytes % 16 == 0,
                "pull: byte count exceeds a buffer or is not a multiple of 16");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
                "pull: 16-byte alignment");
    void* dev_src = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&dev_src, src.data_ptr(), 0) == hipSuccess && dev_src != nullptr,
                "pull: pinned host image is not mapped into the GPU address space");
    any_device_ = true;
    Action a{dls::PULL, (int)stream};
    a.dst = dst.data_ptr();
    a.src = dev_src;
    a.bytes = bytes;
    a.blocks = (int)blocks;
    a.tensor = src;  // keep the host image alive
    acts_.push_back(a);
  }
  void add_memcpy(const at::Tensor& dst, const at::Tensor& src, int64_t bytes, int64_t stream) {
    TORCH_CHECK(dst.nbytes() >= (size_t)bytes && src.nbytes() >= (size_t)bytes, "memcpy: byte count exceeds a buffer");
    any_device_ = true;
    Action a{dls::MEMCPY, (int)stream};
    a.dst = dst.data_ptr();
    a.src = src.data_ptr();
    a.bytes = bytes;
    a.tensor = src;
    acts_.push_back(a);
  }
  void add_memset(const at::Tensor& dst, int64_t value, int64_t stream) {
    any_device_ = true;
    Action a{dls::MEMSET, (int)stream};
    a.dst = dst.data_ptr();
    a.bytes = dst.nbytes();
    a.value = (int)value;
    acts_.push_back(a);
  }
  // runner-owned events, addressed by index (created on first use)
  void add_event_record(int64_t ev, int64_t stream) { acts_.push_back(event_action(dls::EV_RECORD, ev, stream)); }
  void add_event_wait(int64_t ev, int64_t stream) { acts_.push_back(event_action(dls::EV_WAIT, ev, stream)); }
  // p2p ops get work indices in the order they are added
  int64_t add_send(const at::Tensor& t, int64_t peer) { return add_p2p(dls::SEND, t, peer); }
  int64_t add_recv(const at::Tensor& t, int64_t peer) { return add_p2p(dls::RECV, t, peer); }
  void add_work_wait(int64_t w) {
    TORCH_CHECK(w >= 0 && w < n_works_, "unknown p2p work ", w);
    Action a{dls::WORK_WAIT};
    a.index = (int)w;
    acts_.push_back(a);
  }
  // the p2p ops added until group_end form one group (one coalesced RCCL launch)
  void add_group_begin() {
    TORCH_CHECK(group_open_ < 0, "nested p2p group");
    group_open_ = n_works_;
    acts_.push_back(Action{dls::GROUP_BEGIN});
  }
  void add_group_end() {
    TORCH_CHECK(group_open_ >= 0, "p2p group end without a begin");
    Action a{dls::GROUP_END};
    a.index = group_open_;  // first work index of the group; a.value = one past the last
    a.value = n_works_;
    group_open_ = -1;
    acts_.push_back(a);
  }
  // CPU backend only: a kernel group has no hipGraph there, the runner calls back
  void add_pycall(py::object fn) {
    Action a{dls::PYCALL};
    a.fn = fn;
    acts_.push_back(a);
  }

  int64_t size() const { return (int64_t)acts_.size(); }

  void run() {
    TORCH_CHECK(group_open_ < 0, "p2p group left open");
    Backend b;
    b.cs = any_device_ ? c10::hip::getCurrentHIPStream().stream() : nullptr;
    b.copy = copy_;
    b.pg = pg_.get();
    b.hub = hub_.get();
    b.hub_rank = hub_rank_;
    b.dev_type = any_device_ ? c10::DeviceType::CUDA : c10::DeviceType::CPU;
    b.events = &events_;
    dls::run_actions(acts_, n_works_, b);
  }

 private:
  Action event_action(ActKind k, int64_t ev, int64_t stream) {
    TORCH_CHECK(ev >= 0 && ev < 4096, "event index");
    if ((size_t)ev >= events_.size()) events_.resize(ev + 1, nullptr);
    if (!events_[ev]) C10_HIP_CHECK(hipEventCreateWithFlags(&events_[ev], hipEventDisableTiming));
    any_device_ = true;
    Action a{k, (int)stream};
    a.index = (int)ev;
    return a;
  }
  int64_t add_p2p(ActKind k, const at::Tensor& t, int64_t peer) {
    Action a{k};
    a.tensor = t;
    a.index = (int)peer;
    a.value = n_works_;
    if (t.is_cuda()) any_device_ = true;
    acts_.push_back(a);
    return n_works_++;
  }

  std::vector<Action> acts_;
  std::vector<hipEvent_t> events_;
  hipStream_t copy_ = nullptr;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  std::shared_ptr<LoopbackHub> hub_;
  int64_t hub_rank_ = 0;
  int n_works_ = 0;
  int group_open_ = -1;
  bool any_device_ = false;
};

// kernel nodes of a captured hipGraph (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()):
// the launches one replay issues
int64_t graph_kernel_nodes(uint64_t graph) {
  size_t n = 0;
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  C10_HIP_CHECK(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) C10_HIP_CHECK(hipGraphGetNodes(g, nodes.data(), &n));
  int64_t k = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    C10_HIP_CHECK(hipGraphNodeGetType(nd, &t));
    if (t == hipGraphNodeTypeKernel) ++k;
  }
  return k;
}

int64_t graph_nodes(uint64_t graph) {
  size_t n = 0;
  C10_HIP_CHECK(hipGraphGetNodes(reinterpret_cast<hipGraph_t>(graph), nullptr, &n));
  return (int64_t)n;
}

}  // namespace

void register_loopback(py::module& m);  // loopback.cpp

void register_runner(py::module& m) {
  register_loopback(m);
  m.def("graph_kernel_nodes", &graph_kernel_nodes);
  m.def("graph_nodes", &graph_nodes);
  py::class_<StepRunner>(m, "StepRunner")
      .def(py::init<>())
      .def("set_process_group", &StepRunner::set_process_group)
      .def("set_copy_stream", &StepRunner::set_copy_stream)
      .def("add_graph", &StepRunner::add_graph)
      .def("add_pull", &StepRunner::add_pull)
      .def("add_memcpy", &StepRunner::add_memcpy)
      .def("add_memset", &StepRunner::add_memset)
      .def("add_event_record", &StepRunner::add_event_record)
      .def("add_event_wait", &StepRunner::add_event_wait)
      .def("add_send", &StepRunner::add_send)
      .def("add_recv", &StepRunner::add_recv)
      .def("add_work_wait", &StepRunner::add_work_wait)
      .def("add_pycall", &StepRunner::add_pycall)
      .def("add_group_begin", &StepRunner::add_group_begin)
      .def("add_group_end", &StepRunner::add_group_end)
      .def("set_loopback", &StepRunner::set_loopback)
      .def("size", &StepRunner::size)
      .def("run", &StepRunner::run, py::call_guard<py::gil_scoped_release>());
}
