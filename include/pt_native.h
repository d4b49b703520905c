/*
 * pt_native.h — native C-ABI of libpt_hip.so underneath the reference boundary.
 *
 * The reference ABI (path_tracer_kernel.h) is one synchronous pass per call on host-visible
 * memory. This API keeps the scene and the accumulation image resident in HBM, renders any
 * number of passes per call on one HIP stream, and exposes what the benchmark and the multi-GPU
 * driver need (tiling, device image pointer, counters, event timing). Every function returns
 * PT_OK (0) or a negative PT_E* code; pt_last_error() describes the last failure.
 */
#ifndef PT_NATIVE_H
#define PT_NATIVE_H

#include "pt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_E_ARG (-1)
#define PT_E_HIP (-2)
#define PT_E_STATE (-3)
#define PT_E_NOMEM (-4)

typedef struct pt_context pt_context;

const char* pt_last_error(void);
/* Numerics helper: the largest float x >= 0 whose correctly rounded sqrtf is <= c (NaN for NaN, -1 when
 * none). The kernels test length(v) > c as dot(v, v) > x (DevConfig: the kill and SSS thresholds and
 * Fresnel's 0.000005f, path_tracer_kernel.cu:460,612-616, fresnel.h:37): the same outcome, no sqrt. */
float pt_sqrt_le_bound(float c);
int pt_device_count(void);

int pt_context_create(int device, pt_context** out);
void pt_context_destroy(pt_context* ctx);

/* Translate reference-layout, host-readable scene structures into the device layout and upload
 * them (relocating triangle.mat, node.triangle_indices, cube-map faces and texture pixels).
 * triangle_num / texture_num < 0: derive them from the BVH leaves / material texture ids. */
int pt_scene_upload(pt_context* ctx, int mesh_num, pt_bvh_node_device** bvh_nodes, pt_triangle* triangles,
                    int triangle_num, int sphere_num, pt_sphere* spheres, pt_cube_map* sky_cube_map,
                    pt_texture_wrapper* mesh_textures, int texture_num, const pt_configuration* config);
/* Device bytes of the resident scene and its node / triangle counts. */
int pt_scene_info(pt_context* ctx, long long* device_bytes, int* node_num, int* triangle_num);
/* The percentage (1-100, default 100) of the occupancy-sized grid this context's pass launches take:
 * with several contexts rendering frames in flight, the rest of the CUs run the other frames
 * (DESIGN.md §6). Results do not depend on it. */
int pt_set_grid_share(pt_context* ctx, int percent);
/* Tolerance mode (default off; -1 = the PT_MEDIUM_BOUND environment variable, "1" = on, for contexts this API
 * creates; the reference ABI's own context ignores the environment and is on only through this call): the
 * persistent kernel pass_kernel_u and the instrumented pass_kernel (trace_step) walk an in-medium segment's
 * meshes with min_t starting at the segment's free-flight distance (1 + 2^-10), which they draw first, instead
 * of infinity. The wavefront schedule ignores it. Not proven bit-exact against the reference
 * walk (a ray grazing a triangle's plane can make Moller-Trumbore's t fall below its box's entry); measured
 * bit-identical on the whole C4 frame and on subsurface_scattering_s/_a. */
int pt_set_medium_bound(pt_context* ctx, int on);
/* Band order of the work queue. The context's pixels are bands of band_rows rows
 * (pt_set_tiling; one context: bands of the whole frame). pt_band_count gives their number and whether
 * the last is partial; pt_set_band_order(order, n) hands out local band order[i] i-th (a permutation
 * that keeps a partial last band last; n = 0 restores the row order); pt_band_cost_enable(1) zeroes
 * and starts per-band ray-segment counters, which pt_band_cost downloads after the context's work.
 * Orders and counters belong to the current tiling and frame size. Results do not depend on them. */
int pt_band_count(pt_context* ctx, int* bands, int* last_partial);
int pt_set_band_order(pt_context* ctx, const int* order, int n);
int pt_band_cost_enable(pt_context* ctx, int on);
int pt_band_cost(pt_context* ctx, unsigned int* out, int n);
/* The pass kernel (and its template configuration) the last render call of this context launched. */
const char* pt_last_kernel(pt_context* ctx);

/* Interactive refit on the device (Core/triangle_mesh.cpp:271-328 + Bvh/bvh.cpp:332-356, which the
 * reference runs on the host over managed memory). pt_mesh_attach keeps mesh `mesh`'s mesh-local
 * triangles (tri_count of them, at tri_start in the scene's triangle array), the boxes of its last
 * build (node_count, the mesh's node count) and that build's transform on the device;
 * pt_mesh_set_transform then re-transforms the mesh's resident triangles and refits its resident node
 * boxes in place by one kernel, without re-uploading the scene: the result equals
 * pt_scene_builder_set_transform's bit for bit. */
int pt_mesh_attach(pt_context* ctx, int mesh, const pt_triangle* local, int tri_start, int tri_count,
                   const pt_bounding_box* init_boxes, int node_count, pt_float3 init_position, pt_float3 init_scale);
int pt_mesh_set_transform(pt_context* ctx, int mesh, pt_float3 position, pt_float3 scale);

/* Frame geometry. The image is width*height float3 (12 B/pixel) + uchar3, device resident.
 * image_device: optional caller-owned device buffer (e.g. a torch tensor used for the RCCL
 * reduce); NULL = the context allocates its own. */
int pt_frame_setup(pt_context* ctx, int width, int height, void* image_device);
/* Own only the rows y with (y / band_rows) % band_count == band_index (multi-GPU tiling). */
int pt_set_tiling(pt_context* ctx, int band_rows, int band_count, int band_index);

/* Render passes first_pass .. first_pass+pass_count-1 (pass_counter semantics of the reference:
 * pass 1 overwrites the image, later passes add). write_u8: 0 never, 1 every pass, 2 last pass.
 * Asynchronous on the context stream. */
int pt_render_passes(pt_context* ctx, const pt_render_camera* cam, const pt_configuration* config,
                     int first_pass, int pass_count, int write_u8);
/* Several frames at once: passes first_pass .. first_pass+pass_count-1 of `frames` frames, frame f seen
 * through cams[f] (each of the frame's width) and summed into images[f] (width*height float3, device),
 * its 8-bit output into images256[f] (device; images256 or an entry may be NULL: none). Frame f is
 * bit-identical to pt_render_passes(cams[f]) on images[f]; the context's tiling applies to every frame.
 * With the single-kernel schedule one launch per batch of passes renders all the frames, so they share
 * one launch's start-up and tail; otherwise they render one after another. Asynchronous.
 * PT_E_ARG when the share's units times `frames` exceed 2^30 (one launch's 32-bit unit numbering), or when
 * two frames share a buffer (every frame's running sum is accumulated at the same time). */
int pt_render_frames(pt_context* ctx, const pt_render_camera* cams, int frames, const pt_configuration* config,
                     int first_pass, int pass_count, int write_u8, float* const* images,
                     unsigned char* const* images256);
/* 8-bit gamma output of the current image for `pass` accumulated passes (after an external reduce). */
int pt_finalize_u8(pt_context* ctx, const pt_configuration* config, int pass);
/* The same for a caller's float image into a caller's 8-bit buffer (device; the frame's size). */
int pt_finalize_u8_image(pt_context* ctx, const pt_configuration* config, int pass, const float* image,
                         unsigned char* image256);
int pt_synchronize(pt_context* ctx);
/* The context's HIP stream (hipStream_t, non-blocking): callers order their own work on it (the
 * multi-GPU frame packs, gathers and finalizes on it, so frames in flight need no host sync). */
void* pt_stream_handle(pt_context* ctx);

int pt_image_download(pt_context* ctx, pt_float3* image, pt_uchar3* image256);
void* pt_image_device_ptr(pt_context* ctx);
void* pt_image256_device_ptr(pt_context* ctx);

/* Counters since the last pt_stats_reset: ray segments (sum of live rays over every trace step,
 * the reference's thread_shrink inputs), BVH nodes visited and triangle tests (instrumented
 * kernel only, see pt_set_instrumented). */
int pt_stats_reset(pt_context* ctx);
int pt_stats(pt_context* ctx, unsigned long long* segments, unsigned long long* nodes, unsigned long long* tris);
/* All counters: [0] segments, [1] nodes, [2] triangle tests, [3] mesh hits, [4] sphere hits,
 * [5] misses, [6] subsurface scatter events ([1..6] instrumented kernel only); [16..47] the
 * PT_UPROF build's profile counters (tools/uprof.py). n <= 64. */
int pt_stats_all(pt_context* ctx, unsigned long long* out, int n);
int pt_set_instrumented(pt_context* ctx, int on);
/* Kernel schedule of a pass (results are bit-identical under both):
 *   PT_SCHEDULE_PERSISTENT  one persistent launch per pass, a path per lane (default)
 *   PT_SCHEDULE_WAVEFRONT   per depth an extend (BVH walk) and a shade launch over ray queues
 * -1 restores the default (environment PT_MODE=wave selects the wavefront). */
#define PT_SCHEDULE_PERSISTENT 0
#define PT_SCHEDULE_WAVEFRONT 1
int pt_set_schedule(pt_context* ctx, int schedule);
int pt_get_schedule(pt_context* ctx); /* the schedule render calls use, or < 0 on error */
/* HIP-event time of the pass kernels since the last pt_stats_reset (on the stream they run on). */
int pt_kernel_time(pt_context* ctx, double* total_ms, int* launches);
/* The same per kernel kind: 0 single-kernel pass, 1 extend (BVH walk), 2 shade, 3 finalize; -1 all. */
int pt_kernel_time_kind(pt_context* ctx, int kind, double* total_ms, int* launches);

/* Diagnostic: evaluate the device transcendentals (which: 0 sincos, 1 exp, 2 log, 3 atan, 4 asin,
 * 5 acos, 6 pow(x,1.85), 7 tan, 8 sqrt & reciprocal) on n host floats; for the bitwise check
 * against the oracle's host restatement. */
int pt_math_eval_device(pt_context* ctx, int which, const float* x, int n, float* out0, float* out1);

#ifdef __cplusplus
}
#endif

#endif /* PT_NATIVE_H */
