// pt_kernels.h — launchers for the kernels in pt_kernels.hip (host side of the library only).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "pt_glm.h"
#include "pt_path.h"
#include "pt_work.h"

#define PT_BLOCK 256
// workgroup size of pass_kernel_u (the persistent unified pass kernel)
#ifndef PT_UBLOCK
#define PT_UBLOCK 256
#endif

namespace pt {

// Which pass kernel a render launches (pt_runtime.cpp pass_choice): leaf size 1, instrumented, the
// scene's reachable features (pt_path.h PT_FEAT_*).
struct PassChoice {
    bool leaf1, stats;
    int feat;
    bool il;  // the inline-leaf copy of the node array exists (every leaf's skip index is the next record)
    bool multi = false;  // a pt_render_frames launch (several frames): pass_kernel_u's MULTI instance
    bool small = false;  // a launch of fewer than PT_SMALL_LAUNCH units (pass_min_waves)
};
// Launches of fewer units than this run the plain kernel at 7 waves instead of 8 (pass_min_waves).
#define PT_SMALL_LAUNCH (1ll << 21)
// whether launch_pass runs pass_kernel_u for this choice (its node array may then be the inline-leaf copy)
bool pass_uses_unified(const PassChoice& pc, int lds_bytes);
// inline-leaf copy of the node array for pass_kernel_u (pt_kernels.hip inline_leaves_kernel)
hipError_t launch_inline_leaves(const float4* nodes, const float4* tri_geom, const int* np, int R, float4* out,
                                hipStream_t stream);
// the cube map's RGBA8 texels as float4 {u8_unit(r), u8_unit(g), u8_unit(b), 0} (DevScene::cube_f)
hipError_t launch_cube_float(const uint8_t* cube, int texels, float4* out, hipStream_t stream);
hipError_t launch_pass(const LaunchParams* params_dev, const PassChoice& pc, int first_pass, int batch_log2,
                       int write_u8, int grid, int lds_bytes, hipStream_t stream);
// frame: the frame of a pt_render_frames launch whose pass radiances are summed into image / image256
hipError_t launch_accumulate(const LaunchParams* params_dev, int units, int first_pass, int batch_log2, int write_u8,
                             hipStream_t stream, int frame, float* image, uint8_t* image256);
// every frame of a pt_render_frames launch at once; ptrs_dev: {images[0..frames), images256[0..frames)} on the device
hipError_t launch_accumulate_frames(const LaunchParams* params_dev, int units, int first_pass, int batch_log2,
                                    int write_u8, int frames, const uint64_t* ptrs_dev, hipStream_t stream);
// src: the running sum the pass is added to (null: P->out.image in place)
hipError_t launch_accumulate_one(const LaunchParams* params_dev, int unit_begin, int unit_end, int pass, int batch_log2,
                                 int j, int write_u8, const float* rad, const float* src, hipStream_t stream);
// order-independent digest of the 32-bit words [begin, end) of p, added into *out (device)
hipError_t launch_digest_words(const void* p, size_t begin, size_t end, unsigned long long* out, hipStream_t stream);
hipError_t launch_extend(const LaunchParams* P, bool gen, bool leaf1, bool stats, int depth, int pass, hipStream_t s);
hipError_t launch_shade(const LaunchParams* P, bool first, bool last, bool stats, int depth, int pass, hipStream_t s);
int shade_grid_waves();
hipError_t launch_finalize(const LaunchParams* P, int units, int pass, int write_u8, int traced, hipStream_t s);
hipError_t launch_u8(const DevConfig& cfg, const float* image, uint8_t* image256, int pixel_count, int pass,
                     hipStream_t stream);
int pass_grid_size(const PassChoice& pc, int lds_bytes);  // lds_bytes: pass_kernel_u's dynamic LDS
std::string pass_kernel_desc(const PassChoice& pc, int lds_bytes);
int env_int(const char* name, int dflt, int lo, int hi);  // clamped integer from the environment
hipError_t launch_material_consts(DevMaterial* mats, int n, float air_n, hipStream_t stream);
hipError_t launch_mesh_refit(const float4* local, int tri_start, int tri_count, const float4* init_nodes, int node_first,
                             int node_count, const ptglm::M4& T, const ptglm::M4& Tn, const ptglm::M4& C,
                             float4* tri_geom, float4* tri_shade, float4* nodes, hipStream_t stream);
hipError_t launch_math_eval(int which, const float* x, int n, float* o0, float* o1, hipStream_t stream);
hipError_t shrink(int* data, int n, int* scratch, int* tile_counts, int* total_dev, int* total_host,
                  hipStream_t stream);

}  // namespace pt
