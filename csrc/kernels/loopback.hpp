// Single-GPU multi-rank loopback transport (loopback.cpp); the pairing logic is dls::P2PMatcher
// (csrc/runtime/p2p_match.h), also run under ASan / TSan by the native selftest.
#pragma once

#include <torch/extension.h>

#include <atomic>
#include <memory>

#include <hip/hip_runtime.h>

#include "../runtime/p2p_match.h"

// Several ranks of one job living in ONE process on ONE GPU (each with its own compute stream,
// each driven by its own host thread) exchange DAG edges through this hub with RCCL's p2p
// semantics: a send / recv is posted from the rank's thread and ordered after the work already
// enqueued on the rank's current stream (a hipEvent recorded at post time); matched sends and
// recvs (FIFO per (src, dst) pair, equal byte counts, like ncclSend / ncclRecv on one
// communicator) are copied on the hub's own stream; ``wait`` makes the CALLER'S STREAM wait for
// the copy (host-blocking only until the peer has posted its half, as a blocking RCCL
// rendezvous would). ``delay_us`` puts a spinning kernel in front of every copy and ``poison``
// fills each receive buffer with 0xFF (bf16 NaN) at post time, so a consumer kernel that is not
// ordered after its transfer reads NaN instead of data, and a producer that overwrites a buffer
// before its send completed corrupts the transfer: the harness checks the executor's stream
// ordering with real device asynchrony. CPU tensors are copied at match time (test backend).
class LoopbackHub {
 public:
  LoopbackHub(int64_t world, double delay_us, bool poison, double timeout_s);
  ~LoopbackHub();

  int64_t post(bool send, const at::Tensor& t, int64_t self, int64_t peer);
  void wait(int64_t id);
  int64_t world() const { return match_.world(); }
  int64_t transfers() { return match_.matched_pairs(); }
  int64_t bytes() const { return bytes_; }
  int64_t outstanding() { return match_.outstanding(); }

 private:
  struct Done {
    hipEvent_t ev = nullptr;
    ~Done();
  };
  struct Op {
    at::Tensor t;
    hipEvent_t ready = nullptr;
    std::shared_ptr<Done> done;
  };
  void copy(Op& s, Op& r);  // runs under the matcher's lock when a send meets its receive

  dls::P2PMatcher<Op> match_;
  double delay_us_;
  bool poison_;
  double timeout_s_;
  std::atomic<int64_t> bytes_{0};
  hipStream_t stream_ = nullptr;
  int device_ = -1;
};
