// Tile configs 38, 39, 40, 41 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(38)
DLS_GLDS_DEFINE(39)
DLS_GLDS_DEFINE(40)
DLS_GLDS_DEFINE(41)
