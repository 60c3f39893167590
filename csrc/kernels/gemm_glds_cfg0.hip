// Tile configs 34, 35, 12 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(34)
DLS_GLDS_DEFINE(35)
DLS_GLDS_DEFINE(12)
