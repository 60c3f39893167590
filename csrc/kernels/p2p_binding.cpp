// Torch-facing bindings of the device-initiated p2p transport (p2p_device.hpp) and the IPC
// handle exchange a multi-process job maps its peers' arenas and mailboxes with. Remote
// addresses travel as plain integers (a peer's pointer is valid in this process only once its
// IPC handle was opened here — or, for ranks sharing one process, directly).
#include <c10/hip/HIPStream.h>
#include <torch/csrc/utils/pybind.h>
#include <torch/extension.h>

#include <string>

#include "kernels.h"
#include "p2p_device.hpp"

namespace {

hipStream_t cur(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

void check_i64(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.numel() >= 1, what, ": a CUDA int64 tensor");
}

void p2p_tick(at::Tensor step) {
  check_i64(step, "p2p_tick step");
  launch_p2p_tick(step.data_ptr<int64_t>(), cur(step));
}

void p2p_notify(int64_t remote_flag, at::Tensor step) {
  check_i64(step, "p2p_notify step");
  TORCH_CHECK(remote_flag != 0 && remote_flag % 8 == 0, "p2p_notify: flag address");
  launch_p2p_notify(reinterpret_cast<int64_t*>(remote_flag), step.data_ptr<int64_t>(), cur(step));
}

unsigned long long* moved_ptr(const c10::optional<at::Tensor>& moved) {
  if (!moved || !moved->defined()) return nullptr;
  TORCH_CHECK(moved->is_cuda() && moved->scalar_type() == at::kLong, "p2p: int64 byte counter");
  return reinterpret_cast<unsigned long long*>(moved->data_ptr<int64_t>());
}

void p2p_pull(int64_t src, at::Tensor dst, at::Tensor ready, int64_t ack_remote, at::Tensor ticket, at::Tensor step,
              at::Tensor err, int64_t timeout_ticks, c10::optional<at::Tensor> moved) {
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "p2p_pull: dst must be a contiguous CUDA region");
  const int64_t bytes = dst.nbytes();
  TORCH_CHECK(bytes % 16 == 0 && src % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "p2p_pull: 16-byte aligned regions of a multiple of 16 bytes (", bytes, ")");
  check_i64(ready, "p2p_pull ready");
  check_i64(step, "p2p_pull step");
  TORCH_CHECK(ticket.is_cuda() && ticket.scalar_type() == at::kInt, "p2p_pull: int32 ticket");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "p2p_pull: int32 error word");
  TORCH_CHECK(ack_remote != 0 && ack_remote % 8 == 0, "p2p_pull: ack address");
  if (bytes == 0) return;
  launch_p2p_pull(reinterpret_cast<const void*>(src), dst.data_ptr(), bytes, ready.data_ptr<int64_t>(),
                  reinterpret_cast<int64_t*>(ack_remote), reinterpret_cast<unsigned*>(ticket.data_ptr<int>()),
                  step.data_ptr<int64_t>(), err.data_ptr<int>(), timeout_ticks, p2p_pull_blocks(bytes), moved_ptr(moved),
                  cur(dst));
}

// rows of the listed experts' ranges in `off` (int32 [E+1], device): gathered through `idx`
// (int32, expert-sorted order -> source row) when given, else copied as compact rows
void p2p_pull_rows(int64_t src, at::Tensor dst, int64_t row_bytes, c10::optional<at::Tensor> idx, at::Tensor off,
                   at::Tensor experts, int64_t max_rows, at::Tensor ready, int64_t ack_remote, at::Tensor ticket,
                   at::Tensor step, at::Tensor err, int64_t timeout_ticks, c10::optional<at::Tensor> moved) {
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "p2p_pull_rows: contiguous CUDA destination");
  TORCH_CHECK(row_bytes > 0 && row_bytes % 16 == 0 && src % 16 == 0, "p2p_pull_rows: 16-B rows");
  TORCH_CHECK(off.is_cuda() && off.scalar_type() == at::kInt, "p2p_pull_rows: int32 offsets");
  TORCH_CHECK(experts.is_cuda() && experts.scalar_type() == at::kInt, "p2p_pull_rows: int32 expert list");
  TORCH_CHECK(dst.nbytes() >= max_rows * row_bytes, "p2p_pull_rows: destination smaller than max_rows rows");
  const int32_t* ip = nullptr;
  if (idx && idx->defined()) {
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kInt, "p2p_pull_rows: int32 row index");
    ip = idx->data_ptr<int32_t>();
  }
  check_i64(ready, "p2p_pull_rows ready");
  check_i64(step, "p2p_pull_rows step");
  launch_p2p_pull_rows(reinterpret_cast<const void*>(src), dst.data_ptr(), row_bytes, ip, off.data_ptr<int32_t>(),
                       experts.data_ptr<int32_t>(), (int)experts.numel(), max_rows, ready.data_ptr<int64_t>(),
                       reinterpret_cast<int64_t*>(ack_remote), reinterpret_cast<unsigned*>(ticket.data_ptr<int>()),
                       step.data_ptr<int64_t>(), err.data_ptr<int>(), timeout_ticks, moved_ptr(moved), cur(dst));
}

// the sends of one program point: one notify launch (p2p_device.hpp)
void p2p_notify_many(const std::vector<int64_t>& flags, at::Tensor step) {
  TORCH_CHECK(!flags.empty() && (int)flags.size() <= kP2PBatch, "p2p_notify_many: 1..", kP2PBatch, " flags");
  check_i64(step, "p2p_notify_many step");
  int64_t* f[kP2PBatch];
  for (size_t i = 0; i < flags.size(); ++i) {
    TORCH_CHECK(flags[i] != 0 && flags[i] % 8 == 0, "p2p_notify_many: flag address");
    f[i] = reinterpret_cast<int64_t*>(flags[i]);
  }
  launch_p2p_notify_many(f, (int)flags.size(), step.data_ptr<int64_t>(), cur(step));
}

void p2p_delay(double us, at::Tensor like) { launch_delay(us, cur(like)); }

void p2p_wait(at::Tensor flag, at::Tensor step, at::Tensor err, int64_t timeout_ticks, int64_t code) {
  check_i64(flag, "p2p_wait flag");
  check_i64(step, "p2p_wait step");
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "p2p_wait: int32 error word");
  launch_p2p_wait(flag.data_ptr<int64_t>(), step.data_ptr<int64_t>(), err.data_ptr<int>(), timeout_ticks,
                  (int)code, cur(flag));
}

// (handle bytes, offset of t's first byte inside the allocation the handle names)
py::tuple ipc_handle(at::Tensor t) {
  TORCH_CHECK(t.is_cuda(), "ipc_handle: a CUDA tensor");
  void* base = nullptr;
  size_t size = 0;
  C10_HIP_CHECK(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t*>(&base), &size, t.data_ptr()));
  hipIpcMemHandle_t h;
  C10_HIP_CHECK(hipIpcGetMemHandle(&h, base));
  const int64_t off = static_cast<char*>(t.data_ptr()) - static_cast<char*>(base);
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), off);
}

int64_t ipc_open(py::bytes handle) {
  std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "ipc_open: handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  void* p = nullptr;
  C10_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void ipc_close(int64_t p) { C10_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(p))); }

// Launch an instantiated hipGraph on `stream` (a raw hipStream_t) with the GIL released: a
// captured step's whole host cost (torch's CUDAGraph.replay also updates RNG offsets the
// executor's graphs never use, under the GIL — which ranks sharing a process contend for).
void graph_launch(int64_t exec, int64_t stream) {
  py::gil_scoped_release nogil;
  C10_HIP_CHECK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream)));
}

}  // namespace

// A stream of its own (hipStreamCreateWithFlags, non-blocking), outside torch's stream pool:
// the pool hands out 32 streams round-robin over the device's hardware queues, so two pool
// streams can share a queue; HIP gives consecutively created streams consecutive queues.
int64_t stream_create() {
  hipStream_t s = nullptr;
  C10_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return reinterpret_cast<int64_t>(s);
}

void register_p2p(py::module& m) {
  m.def("stream_create", &stream_create);
  m.def("p2p_tick", &p2p_tick);
  m.def("p2p_notify", &p2p_notify);
  m.def("p2p_pull", &p2p_pull, py::arg("src"), py::arg("dst"), py::arg("ready"), py::arg("ack_remote"),
        py::arg("ticket"), py::arg("step"), py::arg("err"), py::arg("timeout_ticks"), py::arg("moved") = py::none());
  m.def("p2p_pull_rows", &p2p_pull_rows, py::arg("src"), py::arg("dst"), py::arg("row_bytes"), py::arg("idx"),
        py::arg("off"), py::arg("experts"), py::arg("max_rows"), py::arg("ready"), py::arg("ack_remote"),
        py::arg("ticket"), py::arg("step"), py::arg("err"), py::arg("timeout_ticks"), py::arg("moved") = py::none());
  m.def("p2p_notify_many", &p2p_notify_many);
  m.def("p2p_wait", &p2p_wait);
  m.def("p2p_delay", &p2p_delay);
  m.def("p2p_pull_blocks", &p2p_pull_blocks);
  m.def("ipc_handle", &ipc_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("graph_launch", &graph_launch);
}
