// Single-GPU multi-rank loopback transport: see loopback.hpp. Used by the executor's Python p2p
// path (parallel/loopback.py) and by the native step runner's SEND / RECV / WORK_WAIT actions
// (runner.cpp, set_loopback), so one GPU exercises exactly the stream ordering an RCCL job
// relies on: the producer's kernels before the send, the transfer, the consumer's kernels after
// the receive, a sent buffer not overwritten before its send completed.
#include "loopback.hpp"

#include <c10/hip/HIPStream.h>
#include <torch/csrc/utils/pybind.h>

#include <chrono>
#include <cstring>

#include "kernels.h"

LoopbackHub::Done::~Done() {
  if (ev) (void)hipEventDestroy(ev);
}

LoopbackHub::LoopbackHub(int64_t world, double delay_us, bool poison, double timeout_s)
    : match_((int)world), delay_us_(delay_us), poison_(poison), timeout_s_(timeout_s) {
  TORCH_CHECK(world >= 1, "loopback: world size");
}

LoopbackHub::~LoopbackHub() {
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
  }
}

int64_t LoopbackHub::post(bool send, const at::Tensor& t, int64_t self, int64_t peer) {
  TORCH_CHECK(t.is_contiguous(), "loopback: p2p buffers must be contiguous");
  Op op;
  op.t = t;
  if (t.is_cuda()) {
    hipStream_t cur = c10::hip::getCurrentHIPStream(t.get_device()).stream();
    if (!send && poison_) C10_HIP_CHECK(hipMemsetAsync(t.data_ptr(), 0xFF, t.nbytes(), cur));
    C10_HIP_CHECK(hipEventCreateWithFlags(&op.ready, hipEventDisableTiming));
    C10_HIP_CHECK(hipEventRecord(op.ready, cur));  // the buffer is ready once cur gets here
  } else if (!send && poison_) {
    std::memset(t.data_ptr(), 0xFF, t.nbytes());
  }
  try {
    return match_.post(send, (int)self, (int)peer, std::move(op), [this](Op& s, Op& r) { copy(s, r); });
  } catch (const std::invalid_argument& e) {
    TORCH_CHECK(false, "loopback: ", e.what());
  }
}

void LoopbackHub::copy(Op& s, Op& r) {
  TORCH_CHECK(s.t.nbytes() == r.t.nbytes(), "loopback: a send of ", s.t.nbytes(), " bytes met a receive of ",
              r.t.nbytes());
  TORCH_CHECK(s.t.is_cuda() == r.t.is_cuda(), "loopback: send and recv on different device kinds");
  auto done = std::make_shared<Done>();
  if (s.t.is_cuda()) {
    if (!stream_) {
      device_ = s.t.get_device();
      C10_HIP_CHECK(hipSetDevice(device_));
      C10_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    }
    C10_HIP_CHECK(hipStreamWaitEvent(stream_, s.ready, 0));
    C10_HIP_CHECK(hipStreamWaitEvent(stream_, r.ready, 0));
    launch_delay(delay_us_, stream_);
    C10_HIP_CHECK(hipMemcpyAsync(r.t.data_ptr(), s.t.data_ptr(), s.t.nbytes(), hipMemcpyDeviceToDevice, stream_));
    C10_HIP_CHECK(hipEventCreateWithFlags(&done->ev, hipEventDisableTiming));
    C10_HIP_CHECK(hipEventRecord(done->ev, stream_));
    (void)hipEventDestroy(s.ready);  // already waited for by the hub stream
    (void)hipEventDestroy(r.ready);
    s.ready = r.ready = nullptr;
  } else {
    std::memcpy(r.t.data_ptr(), s.t.data_ptr(), s.t.nbytes());
  }
  s.done = r.done = done;
  bytes_ += (int64_t)s.t.nbytes();
}

void LoopbackHub::wait(int64_t id) {
  Op op;
  if (!match_.wait(id, timeout_s_, &op)) {
    int self = -1, peer = -1;
    bool send = false;
    match_.describe(id, &self, &peer, &send);
    TORCH_CHECK(false, "loopback: rank ", self, "'s ", send ? "send to " : "recv from ", peer,
                " was never matched within ", timeout_s_, " s (mismatched or deadlocked p2p program)");
  }
  if (op.t.is_cuda() && op.done && op.done->ev) {
    hipStream_t cur = c10::hip::getCurrentHIPStream(op.t.get_device()).stream();
    C10_HIP_CHECK(hipStreamWaitEvent(cur, op.done->ev, 0));  // stream-side, as RCCL's work.wait()
  }
}

void register_loopback(py::module& m) {
  py::class_<LoopbackHub, std::shared_ptr<LoopbackHub>>(m, "LoopbackHub")
      .def(py::init<int64_t, double, bool, double>(), py::arg("world"), py::arg("delay_us") = 0.0,
           py::arg("poison") = true, py::arg("timeout_s") = 120.0)
      .def("post", &LoopbackHub::post, py::arg("send"), py::arg("tensor"), py::arg("rank"), py::arg("peer"))
      .def("wait", &LoopbackHub::wait, py::call_guard<py::gil_scoped_release>())
      .def("outstanding", &LoopbackHub::outstanding)
      .def_property_readonly("world", &LoopbackHub::world)
      .def_property_readonly("transfers", &LoopbackHub::transfers)
      .def_property_readonly("bytes", &LoopbackHub::bytes);
}
