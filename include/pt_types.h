/*
 * pt_types.h — plain-C restatement of the reference's POD data model as it crosses the
 * drop-in boundary (x64 layouts; CUDA float2 is 8-byte aligned).
 *
 * Every struct here is byte-compatible with the reference type it replaces, so a caller
 * built against the reference headers can hand its buffers to this library unchanged.
 * Offsets are asserted below and in tests/test_abi.py.
 *
 *   pt_float3 / pt_float2 / pt_uchar3  <- CUDA float3 / float2 (__align__(8)) / uchar3
 *   pt_ray               <- Core/ray.h:9-18                       (24 B)
 *   pt_scattering        <- Core/material.h:17-29                 (24 B)
 *   pt_medium            <- Core/material.h:31-47                 (32 B)
 *   pt_material          <- Core/material.h:49-78                 (84 B)
 *   pt_sphere            <- Core/sphere.h:11-16                   (100 B)
 *   pt_triangle          <- Core/triangle.h:10-25                 (104 B)
 *   pt_bounding_box      <- Bvh/bounding_box.h:7-10               (36 B)
 *   pt_bvh_node_device   <- Bvh/bvh_node.h:41-47                  (56 B)
 *   pt_render_camera     <- Core/camera.h:14-23                   (64 B)
 *   pt_configuration     <- Core/configuration.h:9-34             (96 B)
 *   pt_cube_map          <- Core/cube_map.h:9-18                  (56 B)
 *   pt_texture_wrapper   <- Core/texture.h:9-13                   (16 B)
 *
 * No torch types, no HIP types: this header is included by the HIP library, by host C++,
 * by the C oracle and (through ctypes mirrors) by Python.
 */
#ifndef PT_TYPES_H
#define PT_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_float3 { float x, y, z; } pt_float3;
typedef struct __attribute__((aligned(8))) pt_float2 { float x, y; } pt_float2;
typedef struct pt_uchar3 { unsigned char x, y, z; } pt_uchar3;

/* Core/ray.h:9-18 */
typedef struct pt_ray {
    pt_float3 origin;
    pt_float3 direction;
} pt_ray;

/* Core/material.h:17-29 */
typedef struct pt_scattering {
    pt_float3 absorption_coefficient;
    pt_float3 reduced_scattering_coefficient;
} pt_scattering;

/* Core/material.h:31-47 */
typedef struct pt_medium {
    float refraction_index;
    float extinction_coefficient;
    pt_scattering scattering;
} pt_medium;

/* Core/material.h:49-78 (C++ bool is one byte on x64) */
typedef struct pt_material {
    pt_float3 diffuse_color;
    pt_float3 emission_color;
    pt_float3 specular_color;
    unsigned char is_transparent;
    float roughness;
    pt_medium medium;
    int diffuse_texture_id;
    int specular_texture_id;
} pt_material;

/* Core/sphere.h:11-16 */
typedef struct pt_sphere {
    pt_float3 center;
    float radius;
    pt_material mat;
} pt_sphere;

/* Core/triangle.h:10-25 ; mat is a pointer into the caller's material array */
typedef struct pt_triangle {
    pt_float3 vertex0, vertex1, vertex2;
    pt_float3 normal0, normal1, normal2;
    pt_float2 uv0, uv1, uv2;
    pt_material* mat;
} pt_triangle;

/* Bvh/bounding_box.h:7-10 */
typedef struct pt_bounding_box {
    pt_float3 left_bottom;
    pt_float3 right_top;
    pt_float3 centroid;
} pt_bounding_box;

/* Bvh/bvh_node.h:41-47 ; triangle_indices points at bvh_leaf_node_triangle_num slots, -1 = empty */
typedef struct pt_bvh_node_device {
    pt_bounding_box box;
    int* triangle_indices;
    unsigned char is_leaf;
    int next_node_index;
} pt_bvh_node_device;

/* Bvh/bvh_node.h:27-39 ; the Morton/CUDA builder's intermediate node (64 B) */
typedef struct pt_bvh_node_morton_code_cuda {
    pt_bounding_box box;
    int left_index;
    int right_index;
    int parent_index;
    unsigned char is_left_leaf;
    unsigned char is_right_leaf;
    unsigned char is_leaf;
    int triangle_index;
    unsigned int morton_code;
    int is_visited;
} pt_bvh_node_morton_code_cuda;

/* Core/camera.h:14-23 */
typedef struct pt_render_camera {
    pt_float3 eye;
    pt_float3 view;
    pt_float3 up;
    pt_float2 resolution;
    pt_float2 fov;
    float aperture_radius;
    float focal_distance;
} pt_render_camera;

/* Bvh/bvh_build_config.h: enum class bvh_build_method (int) */
enum pt_bvh_build_method {
    PT_BVH_NAIVE_CPU = 0,
    PT_BVH_MORTON_CODE_CPU = 1,
    PT_BVH_MORTON_CODE_CUDA = 2,
    /* not a reference method: a binned true-surface-area tree (pt_bvh_build_sah; its GPU twin pt_bvh_build_sah_device),
     * flattened like the others; the closest hit may differ from the reference tree's where visit order decides it
     * (ties, grazed boxes): a stated-tolerance mode, DESIGN.md §5 */
    PT_BVH_SAH = 3
};

/* Core/configuration.h:9-34 */
typedef struct pt_configuration {
    int width;
    int height;
    unsigned char use_fullscreen;
    int block_size;
    int max_block_size;
    int max_tracer_depth;
    float vector_bias_length;
    float energy_exist_threshold;
    float sss_threshold;
    unsigned char use_sky_box;
    unsigned char use_sky;
    unsigned char use_bilinear;
    unsigned char gamma_correction;
    unsigned char use_anti_alias;
    float fov;
    int bvh_leaf_node_triangle_num;
    int bvh_bucket_max_divide_internal_num;
    int bvh_build_block_size;
    int bvh_build;
    float air_refraction_index;
    pt_float3 air_absorption_coef;
    pt_float3 air_reduced_scattering_coef;
    unsigned char cuda_acceleration;
} pt_configuration;

/* Core/cube_map.h:9-18 ; faces are RGBA8, top row first, length x length */
typedef struct pt_cube_map {
    unsigned char* m_x_positive_map;
    unsigned char* m_x_negative_map;
    unsigned char* m_y_positive_map;
    unsigned char* m_y_negative_map;
    unsigned char* m_z_positive_map;
    unsigned char* m_z_negative_map;
    int length;
} pt_cube_map;

/* Core/texture.h:9-13 ; RGBA8, top row first */
typedef struct pt_texture_wrapper {
    int width;
    int height;
    unsigned char* pixels;
} pt_texture_wrapper;

#ifdef __cplusplus
}  /* extern "C" */
#endif

#if defined(__cplusplus)
#define PT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define PT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

PT_STATIC_ASSERT(sizeof(pt_ray) == 24, "ray layout");
PT_STATIC_ASSERT(sizeof(pt_scattering) == 24, "scattering layout");
PT_STATIC_ASSERT(sizeof(pt_medium) == 32, "medium layout");
PT_STATIC_ASSERT(sizeof(pt_material) == 84, "material layout");
PT_STATIC_ASSERT(offsetof(pt_material, roughness) == 40, "material.roughness");
PT_STATIC_ASSERT(offsetof(pt_material, medium) == 44, "material.medium");
PT_STATIC_ASSERT(offsetof(pt_material, diffuse_texture_id) == 76, "material.diffuse_texture_id");
PT_STATIC_ASSERT(sizeof(pt_sphere) == 100, "sphere layout");
PT_STATIC_ASSERT(sizeof(pt_triangle) == 104, "triangle layout");
PT_STATIC_ASSERT(offsetof(pt_triangle, uv0) == 72, "triangle.uv0");
PT_STATIC_ASSERT(offsetof(pt_triangle, mat) == 96, "triangle.mat");
PT_STATIC_ASSERT(sizeof(pt_bvh_node_device) == 56, "bvh_node_device layout");
PT_STATIC_ASSERT(offsetof(pt_bvh_node_device, triangle_indices) == 40, "bvh_node.triangle_indices");
PT_STATIC_ASSERT(offsetof(pt_bvh_node_device, next_node_index) == 52, "bvh_node.next");
PT_STATIC_ASSERT(sizeof(pt_bvh_node_morton_code_cuda) == 64, "bvh_node_morton_code_cuda layout");
PT_STATIC_ASSERT(offsetof(pt_bvh_node_morton_code_cuda, is_left_leaf) == 48, "morton_node.is_left_leaf");
PT_STATIC_ASSERT(offsetof(pt_bvh_node_morton_code_cuda, triangle_index) == 52, "morton_node.triangle_index");
PT_STATIC_ASSERT(sizeof(pt_render_camera) == 64, "render_camera layout");
PT_STATIC_ASSERT(offsetof(pt_render_camera, resolution) == 40, "render_camera.resolution");
PT_STATIC_ASSERT(sizeof(pt_configuration) == 96, "configuration layout");
PT_STATIC_ASSERT(offsetof(pt_configuration, air_refraction_index) == 64, "configuration.air_n");
PT_STATIC_ASSERT(offsetof(pt_configuration, cuda_acceleration) == 92, "configuration.cuda");
PT_STATIC_ASSERT(sizeof(pt_cube_map) == 56, "cube_map layout");
PT_STATIC_ASSERT(sizeof(pt_texture_wrapper) == 16, "texture_wrapper layout");

#endif /* PT_TYPES_H */
