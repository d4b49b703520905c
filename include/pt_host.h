/*
 * pt_host.h — host-side surface around the render call (C-ABI): BVH builder, scene assembly
 * into the reference's data layout, and the orbit camera.
 *
 * These replace the host pieces a reference caller links against:
 *   pt_bvh_build          <- bvh_morton_code_cuda::build_bvh + build_bvh_device_data
 *                            (Bvh/bvh.cpp:862-1047, :244-330); default builder per
 *                            res/configuration/config.json:20 ("MortonCodeCUDA")
 *   pt_scene_builder_*    <- scene_parser::create_scene_data_device (Core/scene_parser.cpp:465-528),
 *                            triangle_mesh::load_obj transform + create_mesh_device_data
 *                            (Core/triangle_mesh.cpp:8-213, :558-655), create_bvh_device_data (:498-540)
 *   pt_view_camera_*      <- view_camera (Core/camera.h:27-80, Core/camera.cpp:3-98)
 *
 * All memory handed out here is ordinary host memory owned by the builder; its pointers are the
 * ones a reference caller would pass to path_tracer_kernel (include/path_tracer_kernel.h).
 */
#ifndef PT_HOST_H
#define PT_HOST_H

#include "pt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- BVH ------------------------------------------------------------------------------------
 * Builds the flattened preorder node array for triangles[0..n) (world space). Leaf triangle ids
 * are start_index + local index, as in the reference. On success *nodes (node_num entries) and
 * *leaf_indices (leaf_num * leaf_size entries, -1 padded) are malloc'd; node[i].triangle_indices
 * points into *leaf_indices. Returns 0 on success. */
int pt_bvh_build(const pt_triangle* triangles, int n, int start_index, int leaf_size, int method,
                 pt_bvh_node_device** nodes, int* node_num, int** leaf_indices, int* leaf_num);
void pt_bvh_free(pt_bvh_node_device* nodes, int* leaf_indices);
/* Any of the three configured builders (pt_bvh_build_method): NaiveCPU = the bucketed "SAH"
 * builder (Bvh/bvh.cpp:16-219, bucket_num = BvhBucketMaxDivideInternalNum); MortonCodeCPU and
 * MortonCodeCUDA = the Morton builder above. Same output contract as pt_bvh_build. */
int pt_bvh_build_ex(const pt_triangle* triangles, int n, int start_index, int leaf_size, int method, int bucket_num,
                    pt_bvh_node_device** nodes, int* node_num, int** leaf_indices, int* leaf_num);
int pt_bvh_build_naive(const pt_triangle* triangles, int n, int start_index, int leaf_size, int bucket_num,
                       pt_bvh_node_device** nodes, int* node_num, int** leaf_indices, int* leaf_num);
/* PT_BVH_SAH (not a reference builder): centroids binned into `bins` bins per axis, splits priced by true surface
 * area, leaves of at most leaf_size triangles, then the reference's preorder flattening. Same output contract. */
int pt_bvh_build_sah(const pt_triangle* triangles, int n, int start_index, int leaf_size, int bins,
                     pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_indices_out, int* leaf_num_out);
/* The same tree built on the HIP device (pt_bvh_sah.hip: one launch per tree level, one workgroup per node), flattened
 * on the host; node arrays byte-equal to pt_bvh_build_sah's. bins 2..64. Returns -3 on a HIP error. */
int pt_bvh_build_sah_device(const pt_triangle* triangles, int n, int start_index, int leaf_size, int bins,
                            pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_indices_out, int* leaf_num_out);

/* Morton helpers exposed for known-answer tests (Bvh/bvh.cpp:370-441). */
unsigned int pt_morton_code(float x, float y, float z);
unsigned int pt_clz_table(unsigned int value);

/* ---- scene assembly ------------------------------------------------------------------------- */
typedef struct pt_scene_builder pt_scene_builder;

typedef struct pt_scene_view {
    int mesh_num;
    pt_bvh_node_device** bvh_nodes;     /* mesh_num pointers, each to that mesh's node array */
    pt_triangle* triangles;
    int triangle_num;
    int sphere_num;
    pt_sphere* spheres;
    pt_cube_map* sky_cube_map;          /* NULL when no background is set */
    pt_texture_wrapper* mesh_textures;  /* NULL when no textures */
    int texture_num;
    pt_material* materials;
    int material_num;
    const int* mesh_node_num;
    const int* mesh_triangle_start;
    const int* mesh_triangle_num;
} pt_scene_view;

pt_scene_builder* pt_scene_builder_create(void);
void pt_scene_builder_destroy(pt_scene_builder* b);
/* Returns the new material's id (index into the mesh material table). */
int pt_scene_builder_add_material(pt_scene_builder* b, const pt_material* m);
int pt_scene_builder_add_sphere(pt_scene_builder* b, pt_float3 center, float radius, const pt_material* m);
/* Object-space triangle soup: vertices/normals tri_num*9 floats, uvs tri_num*6 floats or NULL,
 * tri_material[tri_num] = material id. Applied as in the reference: rotate Z then Y then X
 * (degrees), then scale, then translate; normals by the inverse transpose, renormalised.
 * Returns the mesh index. */
int pt_scene_builder_add_mesh(pt_scene_builder* b, int tri_num, const float* vertices, const float* normals,
                              const float* uvs, const int* tri_material, pt_float3 position, pt_float3 scale,
                              pt_float3 rotate_degrees);
/* faces: 6 * length * length RGBA8 texels, order x+, x-, y+, y-, z+, z-, top row first. */
int pt_scene_builder_set_cube_map(pt_scene_builder* b, int length, const unsigned char* faces);
int pt_scene_builder_add_texture(pt_scene_builder* b, int width, int height, const unsigned char* rgba);
/* Builds every mesh BVH and fixes up the embedded pointers. */
int pt_scene_builder_build(pt_scene_builder* b, int leaf_size, int method);
int pt_scene_builder_build_ex(pt_scene_builder* b, int leaf_size, int method, int bucket_num);
/* Where MortonCodeCUDA builds run: -2 (default) the current HIP device when one is present, else the
 * host builder (identical output); -1 always the host; >= 0 the HIP device (include/pt_bvh.h). */
int pt_scene_builder_set_bvh_device(pt_scene_builder* b, int device);
int pt_scene_builder_view(pt_scene_builder* b, pt_scene_view* out);

/* ---- interactive edits (Core/triangle_mesh.cpp:271-426, Bvh/bvh.cpp:332-356) ------------------
 * set_transform: triangle_mesh::set_transform_device + update_bvh — the mesh's triangles become
 *   translate(position) * scale(scale) of its mesh-local triangles and its node boxes are refitted by
 *   (transform * initial_transform) applied to the corners of its last build (no rebuild).
 * set_rotate + apply_rotate: the mesh-local triangles are rotated by the change of rotation and the
 *   mesh's BVH is rebuilt (node arrays may move: fetch the view again).
 * mesh_local: what pt_mesh_attach (pt_native.h) needs to refit the mesh on a device itself. */
int pt_scene_builder_set_transform(pt_scene_builder* b, int mesh, pt_float3 position, pt_float3 scale);
int pt_scene_builder_set_rotate(pt_scene_builder* b, int mesh, pt_float3 rotate);
int pt_scene_builder_apply_rotate(pt_scene_builder* b, int mesh);
int pt_scene_builder_mesh_local(pt_scene_builder* b, int mesh, const pt_triangle** local, int* tri_start,
                                int* tri_count, const pt_bounding_box** init_boxes, int* node_count,
                                pt_float3* init_position, pt_float3* init_scale);

/* ---- camera (Core/camera.cpp) --------------------------------------------------------------- */
typedef struct pt_view_camera {
    pt_float3 center;
    float yaw, pitch, radius;
    float aperture_radius, focal_distance;
    pt_float2 resolution;
    pt_float2 fov;
} pt_view_camera;

void pt_view_camera_default(pt_view_camera* c);                         /* camera.cpp:3-14 */
void pt_view_camera_set_resolution(pt_view_camera* c, float w, float h); /* camera.cpp:62-66 */
void pt_view_camera_set_fov(pt_view_camera* c, float fov_x);             /* camera.cpp:56-60 */
void pt_view_camera_get_render_camera(const pt_view_camera* c, pt_render_camera* out); /* :80-98 */

/* Reference defaults of res/configuration/config.json + config_parser (Core/config_parser.h:68-100). */
void pt_configuration_default(pt_configuration* cfg);

#ifdef __cplusplus
}
#endif

#endif /* PT_HOST_H */
