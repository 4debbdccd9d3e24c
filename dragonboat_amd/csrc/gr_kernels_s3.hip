// gr_kernels_s3.hip — the step kernels for groups of up to 3 remote slots (gr_kernels.h).
#include "gr_kernels.h"

GR_INSTANTIATE_SLOTS(3)
