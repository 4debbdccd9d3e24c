// gr_kernels_s8.hip — the step kernels for groups of up to 8 remote slots (gr_kernels.h).
#include "gr_kernels.h"

GR_INSTANTIATE_SLOTS(8)
