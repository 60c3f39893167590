// Single-GPU multi-rank loopback transport (loopback.cpp).
#pragma once

#include <torch/extension.h>

#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>

#include <hip/hip_runtime.h>

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
  int64_t world() const { return world_; }
  int64_t transfers() const { return transfers_; }
  int64_t bytes() const { return bytes_; }
  int64_t outstanding();

 private:
  struct Done {
    hipEvent_t ev = nullptr;
    ~Done();
  };
  struct Op {
    bool send = false;
    at::Tensor t;
    int self = 0, peer = 0;
    hipEvent_t ready = nullptr;
    std::shared_ptr<Done> done;
    bool matched = false;
  };
  void match(Op& s, Op& r);

  int64_t world_;
  double delay_us_;
  bool poison_;
  double timeout_s_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::pair<int, int>, std::deque<int64_t>> sends_, recvs_;  // unmatched, by (src, dst)
  std::unordered_map<int64_t, Op> ops_;
  int64_t next_ = 0;
  int64_t transfers_ = 0, bytes_ = 0;
  hipStream_t stream_ = nullptr;
  int device_ = -1;
};
