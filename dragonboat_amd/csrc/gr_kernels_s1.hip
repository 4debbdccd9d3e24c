// gr_kernels_s1.hip — the step kernels for groups of up to 1 remote slots (gr_kernels.h).
#include "gr_kernels.h"

GR_INSTANTIATE_SLOTS(1)
