// pt_kernels.h — launchers for the kernels in pt_kernels.hip (host side of the library only).
#pragma once

#include <hip/hip_runtime.h>

#include "pt_path.h"

#define PT_BLOCK 256

namespace pt {

hipError_t launch_pass(const DevScene& sc, const DevConfig& cfg, const DevCamera& cam, const DevTiling& til,
                       const DevOutput& out, int pass, int write_u8, int grid, bool stats, hipStream_t stream);
hipError_t launch_u8(const DevConfig& cfg, const float* image, uint8_t* image256, int pixel_count, int pass,
                     hipStream_t stream);
int pass_grid_size(bool leaf1, bool stats);
hipError_t launch_math_eval(int which, const float* x, int n, float* o0, float* o1, hipStream_t stream);
hipError_t shrink(int* data, int n, int* scratch, int* tile_counts, int* total_dev, int* total_host,
                  hipStream_t stream);

}  // namespace pt
