// Tile configs 22, 23, 24, 25, 26, 27 of the LDS-DMA GEMM (gemm_glds_impl.h).
#include "gemm_glds_impl.h"

DLS_GLDS_DEFINE(22)
DLS_GLDS_DEFINE(23)
DLS_GLDS_DEFINE(24)
DLS_GLDS_DEFINE(25)
DLS_GLDS_DEFINE(26)
DLS_GLDS_DEFINE(27)
