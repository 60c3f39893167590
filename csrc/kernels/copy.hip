// Host -> HBM parameter refills pulled by a kernel: the workgroups read the pinned host image
// (mapped into the GPU's address space) with 16-byte loads, several in flight per lane, and
// write the arena region. A kernel on the compute stream keeps the refill in stream order
// (hipGraph-capturable like any kernel) and sizes its own PCIe request concurrency, instead
// of the DMA engine path of hipMemcpyAsync.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void host_pull_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                        int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i);
    const u32x4 b = __builtin_nontemporal_load(src + i + stride);
    const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    const u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

}  // namespace

void launch_host_pull(const void* src, void* dst, int64_t bytes, int blocks, hipStream_t stream) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0) return;
  int64_t need = (n16 + 255) / 256;
  int g = (int)(need < blocks ? need : blocks);
  host_pull_kernel<<<g, 256, 0, stream>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst), n16);
}

namespace {

// One wave that spins for ``ticks`` of the 100 MHz constant clock (wall_clock64): the
// single-GPU loopback transport (loopback.cpp) puts it in front of every transfer so that a
// consumer which does not wait for the transfer's event reads the poisoned buffer, not data.
__global__ __launch_bounds__(64) void delay_kernel(int64_t ticks) {
  const int64_t t0 = (int64_t)wall_clock64();
  while ((int64_t)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace

void launch_delay(double us, hipStream_t stream) {
  if (us <= 0) return;
  const int64_t ticks = (int64_t)(us * 100.0);  // wall_clock64 counts at 100 MHz
  delay_kernel<<<1, 64, 0, stream>>>(ticks < 100000000 ? ticks : 100000000);  // at most 1 s
}
