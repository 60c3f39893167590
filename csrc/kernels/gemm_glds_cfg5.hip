// Tile configs 16, 17, 18, 19, 20, 21 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(16)
DLS_GLDS_DEFINE(17)
DLS_GLDS_DEFINE(18)
DLS_GLDS_DEFINE(19)
DLS_GLDS_DEFINE(20)
DLS_GLDS_DEFINE(21)
