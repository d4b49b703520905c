// pt_scene.h — the device-resident scene layout and kernel parameter blocks.
//
// The reference keeps AoS structs in managed memory with embedded pointers (triangle.mat,
// bvh_node_device.triangle_indices, the per-mesh bvh_node_device** table, cube_map face
// pointers, texture_wrapper.pixels). Here everything is relocated into a
// handful of hipMalloc'd arrays addressed by 32-bit indices:
//
//   nodes      float4[2*N]  node i = {lb.xyz, next_node_index (int bits)},
//                                    {rt.xyz, leaf ? leaf_slot : -1 (int bits)}   32 B/node
//              all meshes concatenated; next indices are absolute; mesh m spans
//              [mesh_range[m].x, mesh_range[m].y)  (reference: bvh_nodes[m][0].next_node_index)
//   leaf_tris  int[L*leaf_size]  triangle ids per leaf, -1 padded (bvh.cpp:296-300)
//              when leaf_size == 1 the slot field holds the triangle id directly
//   nodes (inline leaves, leaf_size == 1; the array pass_kernel_u walks, built by inline_leaves_kernel
//              from nodes + tri_geom and handed over in LaunchParams.sc): an internal node as above, a
//              leaf two records {lb.xyz, e2.z}, {rt.xyz, triangle id}, {v0.xyz, e1.x}, {e1.yz, e2.xy}
//              (its next index is the record after them); 32 B/internal node + 64 B/leaf
//   tri_geom   float4[3*T]  {v0.xyz, -}, {v1-v0}, {v2-v0}                       48 B/tri
//   tri_shade  float4[4*T]  {n0.xyz, n1.x}, {n1.yz, n2.xy}, {n2.z, uv0.xy, uv1.x},
//                           {uv1.y, uv2.xy, material id (int bits)}             64 B/tri
//   spheres    float4[2*S]  {center.xyz, radius}, {material id, -, -, -}
//   materials  DevMaterial[M] (96 B), sphere materials appended after mesh materials
//   textures   int4[K] {width, height, byte offset, -} + one RGBA8 byte pool
//   cube       RGBA8, 6 faces back to back (x+, x-, y+, y-, z+, z-), length^2 texels each
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
struct alignas(16) float4 { float x, y, z, w; };
struct alignas(8) int2 { int x, y; };
struct alignas(16) int4 { int x, y, z, w; };
struct alignas(16) uint4 { unsigned int x, y, z, w; };
#endif

namespace pt {

struct alignas(16) DevMaterial {
    float diffuse[3];
    float roughness;
    float emission[3];
    float refraction_index;
    float specular[3];
    float extinction_coefficient;
    float absorption[3];
    float reduced_scattering[3];
    int is_transparent;
    int diffuse_texture_id;
    int specular_texture_id;
    // per-material constants of the shading math, computed on the device by material_consts_kernel
    // with the same functions shade_hit would call (so the values are the ones it would compute):
    float rough_alpha;  // pow(roughness, 1.85) * 0.238 (path_tracer_kernel.cu:571)
    float tir_front;    // asin(n / air_n): fresnel.h:34 TIR threshold entering the material
    float tir_back;     // asin(air_n / n): the same leaving it (transparent back face)
    float ratio_front;  // air_n / n: refraction's in_n / out_n entering (path_tracer_kernel.cu:60)
    float ratio_back;   // n / air_n: the same leaving it
    int spec_zero;      // specular == (0, 0, 0): a reflection's throughput is thr * (0 * shadow) (shade_hit)
};
static_assert(sizeof(DevMaterial) == 112, "DevMaterial layout");

struct DevScene {
    const float4* nodes;
    const int* leaf_tris;
    const int2* mesh_range;
    const float4* tri_geom;
    const float4* tri_shade;
    const float4* spheres;
    const DevMaterial* materials;
    const int4* tex_desc;
    const uint8_t* tex_pool;
    const uint8_t* cube;
    int mesh_num;
    int sphere_num;
    int leaf_size;
    int cube_len;
    int node_count;  // records in `nodes` (2 float4 each); bounds of the node buffer descriptor
    int tri_count;   // records in `tri_geom` (3 float4 each)
    int material_num;  // records in `materials`
    int first_mesh;    // first mesh with a non-empty node range (mesh_num if none) and that range:
    int2 first_range;  //   where every trace step's mesh walk starts
    int nested;        // 1: every node's box contains its children's boxes
    // the cube map's texels as floats {b / 255} per channel (u8_unit, the same values the RGBA8 lookup
    // computes per sample), 6 faces back to back like `cube`; null: the lookup converts the bytes
    const float4* cube_f;
};

// The subset of Core/configuration.h:9-34 that the kernel reads.
struct DevConfig {
    int max_depth;
    float bias;
    float energy_threshold;
    float sss_threshold;
    int use_sky_box;
    int use_sky;
    int use_bilinear;
    int gamma_correction;
    int use_anti_alias;
    float air_n;
    float air_absorption[3];
    float air_reduced_scattering[3];
    // length(v) > threshold tested as dot(v, v) > bound (and length(v) <= threshold as dot(v, v) <= bound)
    // without the square root: bound is the largest float whose correctly rounded square root is <= the
    // threshold (sqrtf is monotone), so each test agrees with its reference form for every v, NaN included
    // (both are false for NaN; the kill test is therefore written !(dot <= bound), pt_path.h alive_after;
    // pt_runtime.cpp sqrt_le_bound, tests/test_abi.py)
    float energy_len2;  // energy_exist_threshold (the kill test, path_tracer_kernel.cu:612-616)
    float sss_len2;     // sss_threshold (:460)
    float refr_len2;    // 0.000005f (fresnel.h:37, length(refraction) <= 0.000005f)
    // pt_set_medium_bound (tolerance mode, off by default): pass_kernel_u (its PT_FEAT_MBOUND instances) and the
    // instrumented pass_kernel (trace_step) walk an in-medium segment's meshes with min_t starting at its
    // free-flight distance (1 + 2^-10) instead of infinity (pt_path.h medium_bound); the wavefront kernels ignore it
    int medium_bound;
};

// Core/camera.h:14-23 plus the per-frame canvas terms generate_ray_kernel derives
// (path_tracer_kernel.cu:337-345): they depend only on the camera, so they are computed once.
struct DevCamera {
    float eye[3];
    float view[3];
    float horizontal[3];
    float vertical[3];
    float x_axis[3];
    float y_axis[3];
    float res_x, res_y;
    float aperture;
    float focal;
};

// Which pixels this launch owns: the frame is cut into bands of band_rows rows dealt
// round-robin over band_count owners; owner band_index takes its share. Single GPU: 1 / 0.
struct DevTiling {
    int width;
    int height;
    int band_rows;
    int band_count;
    int band_index;
    int unit_count;  // pixels owned
    // optional: band_order[i] = the local band the i-th band of units covers (a permutation that keeps
    // a partial last band last; pt_set_band_order), band_cost[b] += ray segments of local band b's
    // finished paths (pt_band_cost_enable). Neither changes a result.
    const int* band_order;
    unsigned int* band_cost;
};

struct DevOutput {
    float* image;            // float3 running sum, reference layout (12 B stride)
    uint8_t* image256;       // uchar3 (3 B stride), may be null
    unsigned int* fetch;     // PT_HEAD_SET work heads of the single-kernel pass (zeroed before launch)
    unsigned long long* stats;  // [0] ray segments, [1..] optional instrumentation
    float* pass_rad;         // batched passes: clamped radiance per (unit, pass) (12 B), summed in order
    int via_rad;             // 1: one-pass launches write pass_rad too (accumulate_kernel adds them afterwards)
    // pt_render_frames: one pass_kernel_u launch renders `frames` frames of the batch (>= 1; 1 otherwise), frame
    // f seen through cams[f]: its units are f * (unit_count << batch_log2) + the unit, its radiances the same
    // range of pass_rad (always via pass_rad), summed into its own image by accumulate_kernel
    int frames;
    const DevCamera* cams;   // frames > 1 only (the launch's `cam` otherwise)
};

// Wavefront queues (pt_wavefront.hip). Ray slots are dense per depth; path state is per pixel.
//   q_o[k][s]  {origin.xyz, pixel (int bits)}     q_d[k][s] {direction.xyz, -}      (k = depth & 1)
//   hit[s]     {t, t1, t2, prim << 2 | type}       type 0 none, 1 sphere, 2 triangle
//   st_thr[px] {throughput.xyz, medium id bits}    st_rad[px] {radiance.xyz, -}
//   counters   [d * PT_SHARDS + k]: rays appended to shard k of the depth-d queue (d >= 1); shard k
//              occupies slots [k * seg_cap, k * seg_cap + count). Depth 0: slot == unit, the units
//              cut into PT_SHARDS regions of seg_cap = ceil(units / PT_SHARDS).
//   heads      PT_HEAD_SET uints per launch of a pass (extend d: 2d, shade d: 2d + 1), pt_work.h
#define PT_SHARDS 8

struct DevWave {
    float4* q_o[2];
    float4* q_d[2];
    float4* hit;       // indexed by the dense ray index of the depth
    float4* st_thr;
    float4* st_rad;
    unsigned int* counters;
    unsigned int* heads;
    int seg_cap;
    int pad;
};

// Everything a pass launch reads, in one device-resident block (pt_runtime.cpp uploads it once per
// render call; kernels take its address as their only pointer argument).
struct LaunchParams {
    DevScene sc;
    DevConfig cfg;
    DevCamera cam;
    DevTiling til;
    DevOutput out;
    DevWave wave;
};

}  // namespace pt
