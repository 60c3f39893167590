// Tile configs 31, 32, 33 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(31)
DLS_GLDS_DEFINE(32)
DLS_GLDS_DEFINE(33)
