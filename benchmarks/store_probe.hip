// Epilogue store-pattern probe (MI355X): 256 workgroups x 512 threads each write one 256 x 256
// bf16 output tile of a [512][ld] matrix — the LM-head GEMM's last phase without its main loop.
//
//   hipcc -O3 --offload-arch=gfx950 benchmarks/store_probe.hip -o build/store_probe && build/store_probe
//
// Modes:
//   0  staged: fragments -> swizzled LDS image -> 16-B row segments (the GEMM's epilogue)
//   1  direct: each lane stores its 8-B fragment pieces (4 columns of a row) straight to memory
//   2  staged + nontemporal stores
//   3  contiguous: each workgroup writes its 128 KiB as one contiguous block (bandwidth ceiling)
//   4  staged, tiles in row-major launch order (blocks of one tile row adjacent)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __bf16 bf16;
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void store_tile(bf16* __restrict__ C, int ldc, int tiles_m) {
  __shared__ bf16x8 smem[8192];  // 128 KiB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / 4, wn = wave % 4;
  int tm, tn;
  if (MODE == 4) {
    tm = blockIdx.x / (gridDim.x / tiles_m);
    tn = blockIdx.x % (gridDim.x / tiles_m);
  } else {
    tm = blockIdx.x % tiles_m;
    tn = blockIdx.x / tiles_m;
  }
  const int m0 = tm * 256, n0 = tn * 256;
  const int g4 = (lane >> 4) * 4, r16 = lane & 15;
  float seed = (float)(blockIdx.x * 7 + lane);
  if (MODE == 3) {
    bf16x8* out = reinterpret_cast<bf16x8*>(C) + (size_t)blockIdx.x * 8192;
    bf16x8 v;
    for (int e = 0; e < 8; ++e) v[e] = (bf16)(seed + e);
    for (int q = tid; q < 8192; q += 512) out[q] = v;
    return;
  }
  if (MODE == 1) {
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wm * 128 + i * 16 + r16, col = n0 + wn * 64 + j * 16 + g4;
        bf16x4 o;
        for (int e = 0; e < 4; ++e) o[e] = (bf16)(seed + i + j + e);
        *reinterpret_cast<bf16x4*>(C + (size_t)row * ldc + col) = o;
      }
    return;
  }
  bf16* img = reinterpret_cast<bf16*>(smem);
  constexpr int BNP = 32;
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 8; ++i) {
      const int cl = wn * 64 + j * 16 + g4, rl = wm * 128 + i * 16 + r16;
      bf16x4 o;
      for (int e = 0; e < 4; ++e) o[e] = (bf16)(seed + i + j + e);
      *reinterpret_cast<bf16x4*>(img + rl * BNP * 8 + (((cl >> 3) ^ (rl & 7)) << 3) + (cl & 7)) = o;
    }
  __syncthreads();
  const bf16x8* img8 = reinterpret_cast<const bf16x8*>(img);
#pragma unroll 4
  for (int q = tid; q < 256 * BNP; q += 512) {
    const int rl = q / BNP, cc = q % BNP;
    const bf16x8 o = img8[rl * BNP + (cc ^ (rl & 7))];
    bf16x8* dst = reinterpret_cast<bf16x8*>(C + (size_t)(m0 + rl) * ldc + n0 + cc * 8);
    if (MODE == 2)
      __builtin_nontemporal_store(o, dst);
    else
      *dst = o;
  }
}

template <int MODE>
float time_mode(bf16* C, int ldc, int tiles_m, int tiles_n, hipEvent_t a, hipEvent_t b) {
  const int grid = tiles_m * tiles_n;
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(store_tile<MODE>, dim3(grid), dim3(512), 0, 0, C, ldc, tiles_m);
  hipEventRecord(a);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(store_tile<MODE>, dim3(grid), dim3(512), 0, 0, C, ldc, tiles_m);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / reps;
}

int main() {
  const int M = 512;
  const int tiles_m = 2, tiles_n = 128;
  const int N = tiles_n * 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int pad : {0, 256}) {
    const int ldc = N + pad;
    bf16* C = nullptr;
    CHECK(hipMalloc(&C, (size_t)M * ldc * 2 + (1 << 20)));
    const double mb = (double)M * N * 2 / 1e6;
    float t0 = time_mode<0>(C, ldc, tiles_m, tiles_n, a, b);
    float t1 = time_mode<1>(C, ldc, tiles_m, tiles_n, a, b);
    float t2 = time_mode<2>(C, ldc, tiles_m, tiles_n, a, b);
    float t3 = time_mode<3>(C, ldc, tiles_m, tiles_n, a, b);
    float t4 = time_mode<4>(C, ldc, tiles_m, tiles_n, a, b);
    CHECK(hipGetLastError());
    printf("ld=%d (%.1f MB): staged %.2f us (%.2f TB/s) | direct %.2f | staged-nt %.2f | contiguous %.2f | "
           "staged row-major %.2f\n",
           ldc, mb, t0, mb / t0 / 1e6 * 1e6 / 1e6, t1, t2, t3, t4);
    CHECK(hipFree(C));
  }
  return 0;
}
