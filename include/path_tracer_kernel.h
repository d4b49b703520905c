/*
 * path_tracer_kernel.h — the drop-in boundary: the reference's own C-ABI for the render call,
 * implemented by libpt_hip.so on MI355X (gfx950).
 *
 *   path_tracer_kernel                  <- Core/path_tracer_kernel.h:18-37
 *                                          (impl. Kernel/path_tracer_kernel.cu:685-780)
 *   path_tracer_kernel_memory_allocate  <- Core/path_tracer_kernel.h:39-46 (impl. :782-796)
 *   path_tracer_kernel_memory_free      <- Core/path_tracer_kernel.h:48-54 (impl. :798-811)
 *   thread_shrink                       <- Core/parallel_function.h:19-22
 *                                          (impl. Kernel/parallel_function.cu:42-49)
 *
 * Same names, argument meaning and error behaviour (void returns; failures print
 * "[Hip]Error ..." and continue, as CUDA_CALL does in Others/utilities.hpp:10-18; the last error
 * is also available from pt_last_error()). Semantics kept:
 *   - pass_counter == 1 overwrites image_pixels, otherwise adds the clamped pass radiance;
 *     image_pixels_256 receives gamma-corrected 8-bit output; row 0 is the top of the image.
 *   - the call is synchronous (ends with a device synchronisation).
 * Differences a caller may observe:
 *   - scene pointers must be host-readable (the reference hands out cudaMallocManaged memory,
 *     which is). The scene is translated into the device layout of DESIGN.md §Data layout and
 *     cached. On pass_counter == 1 (the reference caller resets the pass counter after every
 *     scene edit, Core/path_tracer.cpp:101-107) the caller's scene bytes are hashed, and a
 *     changed digest or pointer re-translates and re-uploads them.
 *   - the per-pixel scratch (not_absorbed / accumulated / rays / energy_exist_pixels /
 *     scatterings) is accepted and ignored: path state lives in registers. memory_allocate
 *     still returns buffers of the reference sizes, allocated as the reference allocates them:
 *     managed memory (hipMallocManaged, host- and device-accessible, path_tracer_kernel.cu:782-796).
 */
#ifndef PATH_TRACER_KERNEL_H
#define PATH_TRACER_KERNEL_H

#include "pt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

void path_tracer_kernel(
    int mesh_num,                              /* in */
    pt_bvh_node_device** bvh_nodes_device,     /* in */
    pt_triangle* triangles_device,             /* in */
    int sphere_num,                            /* in */
    pt_sphere* spheres_device,                 /* in */
    int pixel_count,                           /* in */
    pt_float3* image_pixels,                   /* in out */
    pt_uchar3* image_pixels_256,               /* in out */
    int pass_counter,                          /* in */
    pt_render_camera* render_camera_device,    /* in */
    pt_cube_map* sky_cube_map_device,          /* in */
    pt_float3* not_absorbed_colors_device,     /* in */
    pt_float3* accumulated_colors_device,      /* in */
    pt_ray* rays_device,                       /* in */
    int* energy_exist_pixels_device,           /* in */
    pt_scattering* scatterings_device,         /* in */
    pt_texture_wrapper* mesh_textures_device,  /* in */
    pt_configuration* config_device            /* in */
);

void path_tracer_kernel_memory_allocate(
    pt_float3** not_absorbed_colors_device,    /* in out */
    pt_float3** accumulated_colors_device,     /* in out */
    pt_ray** rays_device,                      /* in out */
    int** energy_exist_pixels_device,          /* in out */
    pt_scattering** scatterings_device,        /* in out */
    int pixel_count                            /* in */
);

void path_tracer_kernel_memory_free(
    pt_float3* not_absorbed_colors_device,
    pt_float3* accumulated_colors_device,
    pt_ray* rays_device,
    int* energy_exist_pixels_device,
    pt_scattering* scatterings_device
);

/* Stable removal of negative entries from a DEVICE int array; returns the new length. */
int thread_shrink(int* energy_exist_pixels_device, int energy_exist_pixels_count);

#ifdef __cplusplus
}
#endif

#endif /* PATH_TRACER_KERNEL_H */
