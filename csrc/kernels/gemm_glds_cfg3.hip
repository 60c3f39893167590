// Tile configs 1, 7, 11, 15 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(1)
DLS_GLDS_DEFINE(7)
DLS_GLDS_DEFINE(11)
DLS_GLDS_DEFINE(15)
