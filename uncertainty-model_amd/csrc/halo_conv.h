// Internal interface of the halo-tiled direct convolution (halo_conv.hip),
// dispatched from igemm_run for the shapes it covers.
#pragma once

#include <hip/hip_runtime.h>

#include "igemm.h"

namespace umamd {

bool halo_applicable(int dtype, const IgArgs& a, int min_tiles, int max_nc);
int halo_run(const IgArgs& a, hipStream_t st);

}  // namespace umamd
