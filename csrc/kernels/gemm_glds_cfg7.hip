// Tile configs 28, 29, 30 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(28)
DLS_GLDS_DEFINE(29)
DLS_GLDS_DEFINE(30)
