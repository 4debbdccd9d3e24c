// gr_kernels_s5.hip — the step kernels for groups of up to 5 remote slots (gr_kernels.h).
#include "gr_kernels.h"

GR_INSTANTIATE_SLOTS(5)
