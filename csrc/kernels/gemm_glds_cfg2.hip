// Tile configs 0, 10, 14 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(0)
DLS_GLDS_DEFINE(10)
DLS_GLDS_DEFINE(14)
