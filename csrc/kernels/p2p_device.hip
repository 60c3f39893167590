// Device-initiated p2p transport kernels — the protocol is in p2p_device.hpp.
//
// Flags are 8-byte words polled by ONE lane with system-scope acquire loads and written with
// system-scope release stores (vector memory instructions; the peer may be another GPU over
// xGMI). Bulk data is pulled by the consumer: its own kernel, on its own stream, reads the
// producer's region after the flag and writes its local region, so the bytes the consumer's
// next kernels read were written by a kernel ordered before them on that stream (a kernel
// boundary then makes them visible to every XCD). The pull kernel starts before the producer
// notifies and touches nothing of the source before the flag, so no stale copy of the source
// can sit in this GPU's caches when it reads.
#include "p2p_device.hpp"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ inline int64_t load_flag(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void store_flag(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane: spin until *flag >= target (100 MHz wall clock bounds it); false on timeout, with
// `code` folded into the error word
__device__ bool spin_ge(const int64_t* flag, int64_t target, int64_t timeout_ticks, int* err, int code) {
  const int64_t t0 = (int64_t)wall_clock64();
  while (load_flag(flag) < target) {
    if ((int64_t)wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__global__ __launch_bounds__(64) void p2p_tick_kernel(int64_t* step) {
  if (threadIdx.x == 0) step[0] = step[0] + 1;
}

__global__ __launch_bounds__(64) void p2p_notify_kernel(int64_t* remote_flag, const int64_t* step) {
  if (threadIdx.x == 0) {
    const int64_t s = step[0];
    __threadfence_system();
    store_flag(remote_flag, s);
  }
}

__global__ __launch_bounds__(256) void p2p_pull_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16, const int64_t* ready, int64_t* ack_remote,
                                                       unsigned* ticket, const int64_t* step, int* err,
                                                       int64_t timeout_ticks) {
  __shared__ int ok;
  const int64_t s = step[0];
  if (threadIdx.x == 0) ok = spin_ge(ready, s, timeout_ticks, err, 1);
  __syncthreads();
  if (ok) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
      const u32x4 a = src[i];
      const u32x4 b = src[i + stride];
      const u32x4 c = src[i + 2 * stride];
      const u32x4 d = src[i + 3 * stride];
      dst[i] = a;
      dst[i + stride] = b;
      dst[i + 2 * stride] = c;
      dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
  }
  __syncthreads();  // every lane's loads of the source have returned (their values were stored)
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1u) % gridDim.x == 0u && ok) store_flag(ack_remote, s);  // the last workgroup: source free
  }
}

__global__ __launch_bounds__(64) void p2p_wait_kernel(const int64_t* flag, const int64_t* step, int* err,
                                                      int64_t timeout_ticks, int code) {
  if (threadIdx.x == 0) spin_ge(flag, step[0], timeout_ticks, err, code);
}

}  // namespace

void launch_p2p_tick(int64_t* step, hipStream_t s) { p2p_tick_kernel<<<1, 64, 0, s>>>(step); }

void launch_p2p_notify(int64_t* remote_flag, const int64_t* step, hipStream_t s) {
  p2p_notify_kernel<<<1, 64, 0, s>>>(remote_flag, step);
}

int p2p_pull_blocks(int64_t bytes) {
  // ~64 KB per workgroup, at most 64 (CUs left to the producer's kernels while it spins)
  const int64_t b = (bytes + 65535) / 65536;
  return (int)(b < 1 ? 1 : (b > 64 ? 64 : b));
}

void launch_p2p_pull(const void* src, void* dst, int64_t bytes, const int64_t* ready, int64_t* ack_remote,
                     unsigned* ticket, const int64_t* step, int* err, int64_t timeout_ticks, int blocks,
                     hipStream_t s) {
  p2p_pull_kernel<<<blocks, 256, 0, s>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), bytes / 16,
                                         ready, ack_remote, ticket, step, err, timeout_ticks);
}

void launch_p2p_wait(const int64_t* flag, const int64_t* step, int* err, int64_t timeout_ticks, int code,
                     hipStream_t s) {
  p2p_wait_kernel<<<1, 64, 0, s>>>(flag, step, err, timeout_ticks, code);
}
