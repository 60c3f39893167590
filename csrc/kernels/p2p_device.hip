// Device-initiated p2p transport kernels — the protocol is in p2p_device.hpp.
//
// Flags are 8-byte words polled by ONE lane with system-scope acquire loads and written with
// system-scope release stores (vector memory instructions; the peer may be another GPU over
// xGMI). Bulk data is pulled by the consumer in two launches on its own stream: a one-wave
// kernel waits for the producer's flag, then a copy kernel reads the producer's region and
// writes the local one. Every load of the source thus belongs to a kernel that STARTED after
// the flag was seen, so the kernel boundary's cache maintenance (not an in-kernel fence, whose
// invalidation reaches only the issuing XCD's caches) orders it after the producer's bytes —
// measured necessary when ranks share one GPU: a single wait-then-copy kernel read source lines
// that a co-running kernel of the producer had pulled into another XCD's L2 before the
// producer wrote them. The consumer's own next kernels read what the copy wrote in stream order.
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

// The copy half of a pull. It is launched AFTER the wait kernel that saw the producer's flag,
// so the kernel boundary between them — not an in-kernel fence — orders every load here after
// the producer's data: a wait and its reads inside ONE kernel could read lines a co-running
// kernel pulled into another XCD's L2 before the producer wrote them (ranks sharing a GPU).
// block `bi` of `nb` copying one region (shared by the single and the batched pulls)
__device__ __forceinline__ void copy_region(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16,
                                            int64_t* ack_remote, unsigned* ticket, int64_t s,
                                            unsigned long long* moved, int bi, int nb) {
  const int64_t stride = (int64_t)nb * 256;
  int64_t i = (int64_t)bi * 256 + threadIdx.x;
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
  __syncthreads();  // every lane's loads of the source have returned (their values were stored)
  if (threadIdx.x == 0) {
    if (moved && bi == 0)
      __hip_atomic_fetch_add(moved, (unsigned long long)n16 * 16u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1u) % (unsigned)nb == 0u) store_flag(ack_remote, s);  // the last workgroup: source free
  }
}

__global__ __launch_bounds__(256) void p2p_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16, int64_t* ack_remote, unsigned* ticket,
                                                       const int64_t* step, unsigned long long* moved) {
  copy_region(src, dst, n16, ack_remote, ticket, step[0], moved, blockIdx.x, gridDim.x);
}

struct FlagBatch {
  const int64_t* flag[kP2PBatch];
  int n;
};

__global__ __launch_bounds__(64) void p2p_notify_many_kernel(FlagBatch b, const int64_t* step) {
  if (threadIdx.x == 0) {
    const int64_t s = step[0];
    __threadfence_system();
    for (int i = 0; i < b.n; ++i) store_flag(const_cast<int64_t*>(b.flag[i]), s);
  }
}

// Routed-row pulls (expert parallelism): only the token rows a routing selected cross the link.
// For each selected expert e (experts[0..n_exp)): rows j in [off[e], off[e+1]) of the
// expert-sorted order; `gather` (idx != nullptr): dst row j <- src row idx[j] (a hidden state
// to the expert's GPU); else dst row j - off[e] <- src row j - off[e] (an expert's compact
// output back). Row counts live on the device (the routing computed there): no host sync.
__global__ __launch_bounds__(256) void p2p_pull_rows_kernel(const char* __restrict__ src, char* __restrict__ dst,
                                                            int64_t row_bytes, const int32_t* __restrict__ idx,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ experts, int n_exp,
                                                            int64_t* ack_remote, unsigned* ticket,
                                                            const int64_t* step, unsigned long long* moved) {
  const int64_t s = step[0];
  const int64_t v16 = row_bytes / 16;  // 16-B vectors per row
  unsigned long long mine = 0;
  {
    for (int q = 0; q < n_exp; ++q) {
      const int e = experts[q];
      const int64_t lo = off[e], hi = off[e + 1];
      const int64_t n = (hi - lo) * v16;
      for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
        const int64_t j = lo + k / v16, c = k % v16;
        const int64_t srow = idx ? idx[j] : j - lo;
        const int64_t drow = idx ? j : j - lo;
        reinterpret_cast<u32x4*>(dst + drow * row_bytes)[c] = reinterpret_cast<const u32x4*>(src + srow * row_bytes)[c];
      }
      if (blockIdx.x == 0 && threadIdx.x == 0) mine += (unsigned long long)(hi - lo) * row_bytes;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (mine && moved) __hip_atomic_fetch_add(moved, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if ((old + 1u) % gridDim.x == 0u) store_flag(ack_remote, s);
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
                     unsigned long long* moved, hipStream_t s) {
  p2p_wait_kernel<<<1, 64, 0, s>>>(ready, step, err, timeout_ticks, 1);
  p2p_copy_kernel<<<blocks, 256, 0, s>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), bytes / 16,
                                         ack_remote, ticket, step, moved);
}

void launch_p2p_wait(const int64_t* flag, const int64_t* step, int* err, int64_t timeout_ticks, int code,
                     hipStream_t s) {
  p2p_wait_kernel<<<1, 64, 0, s>>>(flag, step, err, timeout_ticks, code);
}

void launch_p2p_pull_rows(const void* src, void* dst, int64_t row_bytes, const int32_t* idx, const int32_t* off,
                          const int32_t* experts, int n_exp, int64_t max_rows, const int64_t* ready,
                          int64_t* ack_remote, unsigned* ticket, const int64_t* step, int* err, int64_t timeout_ticks,
                          unsigned long long* moved, hipStream_t s) {
  const int blocks = p2p_pull_blocks(max_rows * row_bytes);
  p2p_wait_kernel<<<1, 64, 0, s>>>(ready, step, err, timeout_ticks, 1);
  p2p_pull_rows_kernel<<<blocks, 256, 0, s>>>(static_cast<const char*>(src), static_cast<char*>(dst), row_bytes, idx,
                                              off, experts, n_exp, ack_remote, ticket, step, moved);
}

void launch_p2p_notify_many(int64_t* const* flags, int n, const int64_t* step, hipStream_t s) {
  FlagBatch b{};
  b.n = n;
  for (int i = 0; i < n; ++i) b.flag[i] = flags[i];
  p2p_notify_many_kernel<<<1, 64, 0, s>>>(b, step);
}
