#pragma once
// The fp16x3 planes of the 7x7 stem's zero-extended weight image, and its bound, in one launch
// (stem_pack.hip).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mpit {

// w: fp32 [Co][R][S][C] (channels_last [Co, C, R, S], C <= 4, R, S <= 8); planes: fp16
// [2][Co][8][8][4] (h, l of the zero-extended image scaled by 2^e, e from max |w|); bound: the
// slotted bound buffer (kBoundFloats fp32, slot 0 = max |w|).
void stem_weight_planes(int dev, hipStream_t s, uintptr_t w, int Co, int C, int R, int S, uintptr_t planes,
                        uintptr_t bound);

}  // namespace mpit
