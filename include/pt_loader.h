/*
 * pt_loader.h — host-side ingestion around the render call (C-ABI): the reference's JSON
 * configuration and scene loaders, its OBJ loader, image decoding and PNG output.
 *
 * These replace the host pieces a reference caller links against:
 *   pt_config_load        <- config_parser::load_config + create_config_device_data
 *                            (Core/config_parser.cpp:8-124, :159-187; keys Core/config_parser.h:14-36)
 *   pt_scene_load         <- scene_parser::load_scene + create_scene_data_device
 *                            (Core/scene_parser.cpp:37-442, :465-528; keys Core/scene_parser.h:23-54)
 *   pt_material_preset    <- the built-in materials (Core/material.cpp:12-577, registered by name in
 *                            Core/scene_parser.cpp:675-708)
 *   pt_obj_load           <- triangle_mesh::load_obj's use of tinyobjloader 1.1.0
 *                            (Core/triangle_mesh.cpp:8-213; lib/tiny_obj_loader/tiny_obj_loader.h:1662-1959)
 *   pt_image_load         <- image_loader::load_image (Others/image_loader.cpp:31-95, FreeImage)
 *   pt_image_write_png    <- the PNG screenshot of the 8-bit framebuffer (Main/window.cpp:712-740)
 *
 * Error convention: 0 on success, a negative code on failure, with the reference's
 * "[Error]..." message printed to stderr.
 */
#ifndef PT_LOADER_H
#define PT_LOADER_H

#include "pt_host.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fills *cfg from a config.json (every value a string). On failure *cfg holds the
 * config_parser class defaults (Core/config_parser.h:71-93). The reference parses "FOV" with
 * parse_bool (config_parser.cpp:111), so cfg->fov is 0 unless the file says "true"; the camera
 * never reads it (it uses 45 degrees, Main/window.cpp:359). */
int pt_config_load(const char* path, pt_configuration* cfg);

/* A built-in material by name ("iron", "glass", "wall_white", "light", ...). */
int pt_material_preset(const char* name, pt_material* out);

/* Triangulated OBJ as loaded by tinyobjloader (triangulate = true): per-triangle corners and
 * normals (triangle_num * 9 floats each), uvs (triangle_num * 6) or NULL when the file has no
 * texcoords, and the shape (group) index of each triangle. */
typedef struct pt_obj_mesh {
    int triangle_num;
    int shape_num;
    int vertex_num;     /* attrib.vertices.size() / 3 */
    float* vertices;
    float* normals;
    float* uvs;
    int* shape_of_triangle;
} pt_obj_mesh;
int pt_obj_load(const char* path, pt_obj_mesh* out);
void pt_obj_free(pt_obj_mesh* mesh);

/* Loads a scene JSON into a builder and builds it (BVH per mesh). Asset paths in the scene are
 * Windows-style and relative to the reference's working directory (the gpu_path_tracer folder):
 * backslashes become '/', and relative paths are taken relative to root_dir (NULL = the current
 * directory). background_override, when non-NULL, replaces the Background's folder
 * (Path + Name) and background_format its Format — for scenes whose skybox is not in the
 * checkout. leaf_size / bvh_method are the configuration's BvhLeafNodeTriangleNum and
 * BvhBuildMethod. */
typedef struct pt_scene_load_options {
    const char* root_dir;
    const char* background_override;
    const char* background_format;
    int leaf_size;
    int bvh_method;
    int bucket_num; /* BvhBucketMaxDivideInternalNum (naive builder) */
} pt_scene_load_options;
int pt_scene_load(pt_scene_builder* builder, const char* scene_path, const pt_scene_load_options* options);

/* RGBA8, top row first, alpha 255 (FreeImage_ConvertTo24Bits then RGBA). *rgba is malloc'd. */
int pt_image_load(const char* path, int* width, int* height, unsigned char** rgba);
void pt_image_free(unsigned char* rgba);
/* JPEG decoding of pt_image_load with a chosen arithmetic (pt_jpeg.cpp): PT_JPEG_IJG9 is libjpeg 9a's
 * fast IDCT and colour tables, what FreeImage 3.17 runs by default and what pt_image_load uses;
 * PT_JPEG_IJG6 is libjpeg 6b's (libjpeg-turbo's), the test hook that pins the shared decoder against
 * PIL. RGBA8, top row first; free with pt_image_free. */
#define PT_JPEG_IJG9 0
#define PT_JPEG_IJG6 1
int pt_jpeg_decode(const unsigned char* data, size_t size, int variant, int* width, int* height, unsigned char** rgba);
/* channels 3 (RGB) or 4 (RGBA), top row first. */
int pt_image_write_png(const char* path, int width, int height, const unsigned char* pixels, int channels);

#ifdef __cplusplus
}
#endif

#endif /* PT_LOADER_H */
