// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (built into oracle/_ref/libptref.so).
//
// Links the third-party code the reference vendors, compiled from where it lies under
// /root/reference/gpu_path_tracer/lib (no copies, no stand-in headers):
//   tinyobjloader 1.1.0   lib/tiny_obj_loader/tiny_obj_loader.cc (+ .h)
//   glm 0.9.9             lib/glm (header-only)
//   lodepng               lib/lodepng/lodepng.cpp (+ .h)
// and drives them exactly as the reference's host code does, so the repository's own host
// ingestion (pathtracerwithcuda_amd/csrc/pt_loader.cpp, pt_host.cpp, pt_image.cpp) can be pinned
// bit for bit against the real libraries instead of against a restatement:
//   ptref_mesh_load   <- Core/triangle_mesh.cpp:8-213 (tinyobj::LoadObj, triangulate = true;
//                        corner gather; glm rotate Z,Y,X + inverse transpose for normals)
//                        followed by Core/triangle_mesh.cpp:625-647 (glm translate * scale,
//                        normals by its inverse transpose), normalize = Math/cuda_math.hpp:1458
//                        with the host rsqrtf of :33-36.
//   ptref_refit       <- Core/triangle_mesh.cpp:271-328 + Bvh/bvh.cpp:332-356 (glm transform, refit)
//   ptref_png_decode  <- lodepng::decode to RGBA8 (the decoder the reference vendors next to
//                        Core/cube_map_loader.h:17).
// Only tests/ link this library; nothing in the product path does.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "glm/glm.hpp"
#include "glm/gtc/matrix_transform.hpp"
#include "lodepng/lodepng.h"
#include "tiny_obj_loader/tiny_obj_loader.h"

namespace {
struct F3 {
    float x, y, z;
};
// Math/cuda_math.hpp:33-36 (host rsqrtf = 1/sqrtf) and :1458-1462 (normalize = v * rsqrtf(dot(v,v)))
F3 ref_normalize(F3 v) {
    const float d = v.x * v.x + v.y * v.y + v.z * v.z;
    const float inv = 1.0f / sqrtf(d);
    return {v.x * inv, v.y * inv, v.z * inv};
}
}  // namespace

extern "C" {

// Loads `path` and applies the reference's mesh transforms. On success returns the triangle count
// and mallocs *vertices / *normals (n*9 floats), *uvs (n*6 floats, zeros without texcoords) and
// *shape_of_triangle (n ints); *has_uv tells whether the file had texcoords. Returns -1 when the
// reference's load_obj would return false (load failure, no normals, non-triangle face).
int ptref_mesh_load(const char* path, const float* position, const float* scale, const float* rotate,
                    float** vertices, float** normals, float** uvs, int** shape_of_triangle, int* has_uv) {
    std::string filename(path);
    const size_t slash = filename.find_last_of('/');
    const std::string base = slash == std::string::npos ? std::string() : filename.substr(0, slash + 1);

    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> materials;
    tinyobj::attrib_t attrib;
    std::string error;
    if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &error, filename.c_str(), base.c_str())) return -1;
    if (attrib.normals.empty()) return -1;
    for (const auto& s : shapes)
        for (auto num : s.mesh.num_face_vertices)
            if (num != 3) return -1;

    glm::mat4 rotate_mat(1.0f);
    rotate_mat = glm::rotate(rotate_mat, glm::radians(rotate[2]), glm::vec3(0.0f, 0.0f, 1.0f));
    rotate_mat = glm::rotate(rotate_mat, glm::radians(rotate[1]), glm::vec3(0.0f, 1.0f, 0.0f));
    rotate_mat = glm::rotate(rotate_mat, glm::radians(rotate[0]), glm::vec3(1.0f, 0.0f, 0.0f));
    const glm::mat4 rotate_it = glm::transpose(glm::inverse(rotate_mat));
    glm::mat4 transform_mat(1.0f);
    transform_mat = glm::translate(transform_mat, glm::vec3(position[0], position[1], position[2]));
    transform_mat = glm::scale(transform_mat, glm::vec3(scale[0], scale[1], scale[2]));
    const glm::mat4 transform_it = glm::transpose(glm::inverse(transform_mat));

    std::vector<float> v, n, t;
    std::vector<int> sh;
    for (size_t i = 0; i < shapes.size(); i++) {
        const auto& mesh = shapes[i].mesh;
        for (size_t f = 0; f < mesh.num_face_vertices.size(); f++) {
            for (int k = 0; k < 3; k++) {
                const tinyobj::index_t idx = mesh.indices[f * 3 + k];
                glm::vec4 p(attrib.vertices[idx.vertex_index * 3], attrib.vertices[idx.vertex_index * 3 + 1],
                            attrib.vertices[idx.vertex_index * 3 + 2], 1.0f);
                glm::vec4 q(attrib.normals[idx.normal_index * 3], attrib.normals[idx.normal_index * 3 + 1],
                            attrib.normals[idx.normal_index * 3 + 2], 0.0f);
                float u0 = 0.0f, u1 = 0.0f;
                // A face corner without a texcoord ("f v//vn") has texcoord_index -1, and the reference
                // reads attrib.texcoords[-2] (:114-127, out of bounds: undefined). Zero is taken there.
                if (!attrib.texcoords.empty() && idx.texcoord_index >= 0) {
                    u0 = attrib.texcoords[idx.texcoord_index * 2];
                    u1 = attrib.texcoords[idx.texcoord_index * 2 + 1];
                }
                // load_obj (:154-166): rotate, normals by the inverse transpose, renormalised
                p = rotate_mat * p;
                q = rotate_it * q;
                F3 nn = ref_normalize({q.x, q.y, q.z});
                // create_mesh_device_data (:625-647): current transform = translate * scale
                glm::vec4 wp = transform_mat * glm::vec4(p.x, p.y, p.z, 1.0f);
                glm::vec4 wq = transform_it * glm::vec4(nn.x, nn.y, nn.z, 0.0f);
                F3 wn = ref_normalize({wq.x, wq.y, wq.z});
                v.insert(v.end(), {wp.x, wp.y, wp.z});
                n.insert(n.end(), {wn.x, wn.y, wn.z});
                t.insert(t.end(), {u0, u1});
            }
            sh.push_back((int)i);
        }
    }
    const int tri = (int)sh.size();
    *vertices = (float*)malloc(v.size() * sizeof(float) + 1);
    *normals = (float*)malloc(n.size() * sizeof(float) + 1);
    *uvs = (float*)malloc(t.size() * sizeof(float) + 1);
    *shape_of_triangle = (int*)malloc(sh.size() * sizeof(int) + 1);
    if (!v.empty()) std::memcpy(*vertices, v.data(), v.size() * sizeof(float));
    if (!n.empty()) std::memcpy(*normals, n.data(), n.size() * sizeof(float));
    if (!t.empty()) std::memcpy(*uvs, t.data(), t.size() * sizeof(float));
    if (!sh.empty()) std::memcpy(*shape_of_triangle, sh.data(), sh.size() * sizeof(int));
    *has_uv = attrib.texcoords.empty() ? 0 : 1;
    return tri;
}

// lodepng::decode to RGBA8, top row first. Returns lodepng's error code (0 = ok).
int ptref_png_decode(const char* path, int* width, int* height, unsigned char** rgba) {
    std::vector<unsigned char> out;
    unsigned w = 0, h = 0;
    const unsigned err = lodepng::decode(out, w, h, std::string(path));
    if (err) return (int)err;
    *width = (int)w;
    *height = (int)h;
    *rgba = (unsigned char*)malloc(out.size() + 1);
    std::memcpy(*rgba, out.data(), out.size());
    return 0;
}

// Core/triangle_mesh.cpp:271-328 (set_transform_device) with update_bvh (Bvh/bvh.cpp:332-356), on glm:
// the transform built as :276-278 (translate then scale), n mesh-local vertices and (normalised) normals
// -> world vertices and renormalised normals; m boxes (lb.xyz, rt.xyz) of the build made under the
// initial transform (ipos, iscl; m_mesh_initial_transform = its inverse, :199-204) -> refitted boxes.
void ptref_refit(const float* ipos, const float* iscl, const float* pos, const float* scl, const float* v,
                 const float* nrm, int n, const float* boxes, int m, float* v_out, float* n_out, float* boxes_out) {
    glm::mat4 initial(1.0f);
    initial = glm::translate(initial, glm::vec3(ipos[0], ipos[1], ipos[2]));
    initial = glm::scale(initial, glm::vec3(iscl[0], iscl[1], iscl[2]));
    const glm::mat4 initial_transform_mat = glm::inverse(initial);
    glm::mat4 transform_mat(1.0f);
    transform_mat = glm::translate(transform_mat, glm::vec3(pos[0], pos[1], pos[2]));
    transform_mat = glm::scale(transform_mat, glm::vec3(scl[0], scl[1], scl[2]));
    const glm::mat4 inverse_transpose_transform_mat = glm::transpose(glm::inverse(transform_mat));
    for (int i = 0; i < n; i++) {
        glm::vec4 p(v[3 * i], v[3 * i + 1], v[3 * i + 2], 1.0f);
        glm::vec4 q(nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2], 0.0f);
        p = transform_mat * p;
        q = inverse_transpose_transform_mat * q;
        const F3 nn = ref_normalize({q.x, q.y, q.z});
        v_out[3 * i] = p.x; v_out[3 * i + 1] = p.y; v_out[3 * i + 2] = p.z;
        n_out[3 * i] = nn.x; n_out[3 * i + 1] = nn.y; n_out[3 * i + 2] = nn.z;
    }
    for (int j = 0; j < m; j++) {
        glm::vec4 lb(boxes[6 * j], boxes[6 * j + 1], boxes[6 * j + 2], 1.0f);
        glm::vec4 rt(boxes[6 * j + 3], boxes[6 * j + 4], boxes[6 * j + 5], 1.0f);
        lb = transform_mat * initial_transform_mat * lb;
        rt = transform_mat * initial_transform_mat * rt;
        boxes_out[6 * j] = lb.x; boxes_out[6 * j + 1] = lb.y; boxes_out[6 * j + 2] = lb.z;
        boxes_out[6 * j + 3] = rt.x; boxes_out[6 * j + 4] = rt.y; boxes_out[6 * j + 5] = rt.z;
    }
}

void ptref_free(void* p) { free(p); }

}  // extern "C"
