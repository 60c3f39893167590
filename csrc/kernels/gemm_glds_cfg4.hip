// Tile configs 2, 6, 3, 4, 5 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(2)
DLS_GLDS_DEFINE(6)
DLS_GLDS_DEFINE(3)
DLS_GLDS_DEFINE(4)
DLS_GLDS_DEFINE(5)
