// Tile configs 8, 9, 13 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(8)
DLS_GLDS_DEFINE(9)
DLS_GLDS_DEFINE(13)
