// Internal interface of the streaming 1x1 convolution (stream1x1.hip),
// dispatched from igemm_run for the high-resolution 1x1 shapes it covers.
#pragma once

#include <hip/hip_runtime.h>

#include "igemm.h"

namespace umamd {

bool stream1x1_applicable(int dtype, const IgArgs& a);
int stream1x1_run(const IgArgs& a, hipStream_t st);
// small-M 1x1 convs (M < 16k pixels, C <= 512): round 6
bool s1x1_small_applicable(int dtype, const IgArgs& a);
int s1x1_small_run(const IgArgs& a, hipStream_t st);

}  // namespace umamd
