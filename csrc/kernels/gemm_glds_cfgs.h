// Per-config entry points of the LDS-DMA GEMM (one function pair per tile config, defined in the
// gemm_glds_cfg*.hip translation units so the 46 configs compile in parallel), and the split-K
// reduce launcher shared by all of them (gemm_glds.hip).
#pragma once
#include "kernels.h"

#define DLS_GLDS_DECLARE(ID)                                                                                    \
  bool glds_launch_cfg##ID(const GemmArgs& a, int splitk, float* ws, hipStream_t s, const float* ln_colsum,     \
                           int ln_mode, float ln_eps, const int* rows, bool persist);                           \
  void glds_grouped_cfg##ID(const GemmArgs& a, int n_groups, const int* offsets, const unsigned long long* w_ptrs, \
                            const unsigned long long* c_ptrs, hipStream_t s, const int* a_rows);
#define DLS_GLDS_ALL(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) \
  X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32) X(33) X(34) X(35) \
  X(36) X(37) X(38) X(39) X(40) X(41) X(42) X(43) X(44) X(45) X(46) X(47)
DLS_GLDS_ALL(DLS_GLDS_DECLARE)

// split-K reduce launch(es) after a GEMM whose partials went to the workspace; true when the
// reduce also wrote a.norm_out
bool glds_reduce(const GemmArgs& a, int splitk, float* ws, hipStream_t s, const float* ln_colsum, int ln_mode,
                 float ln_eps, const int* rows, const Epi& ep);
