// san_driver.cpp — host-only driver of the ingestion layer for the ASan + UBSan build (tools/san/Makefile,
// tests/test_sanitizers.py). It links the host sources (pt_loader.cpp, pt_image.cpp, pt_host.cpp) with
// -fsanitize=address,undefined and runs them over the files named on the command line: the reference's
// own fixtures and corrupted copies of them. Loader failures are expected on corrupted inputs; only a
// sanitizer report or a crash fails the run.
//
//   san_driver config FILE... | obj FILE... | image OUT.png FILE... | scene ROOT SCENE [BG FMT] | bvh SEED
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/pt_bvh.h"
#include "../../include/pt_host.h"
#include "../../include/pt_loader.h"
#include "../../include/pt_native.h"

// This build has no HIP runtime: no device, so MortonCodeCUDA scenes take the host builder.
extern "C" int pt_device_count(void) { return 0; }
extern "C" int pt_bvh_build_device(const pt_triangle*, int, int, int, pt_bvh_node_device**, int*, int**, int*) {
    return -1;
}
extern "C" int pt_bvh_build_sah_device(const pt_triangle*, int, int, int, int, pt_bvh_node_device**, int*, int**, int*) {
    return -1;
}

static int run_scene(const char* root, const char* scene, const char* bg, const char* fmt) {
    for (int method = 0; method < 4; method++) {  // NaiveCPU, MortonCodeCPU, MortonCodeCUDA, PT_BVH_SAH
        for (int leaf = 1; leaf <= 3; leaf += 2) {
            pt_scene_builder* b = pt_scene_builder_create();
            pt_scene_load_options o;
            std::memset(&o, 0, sizeof(o));
            o.root_dir = root;
            o.background_override = bg;
            o.background_format = fmt;
            o.leaf_size = leaf;
            o.bvh_method = method;
            o.bucket_num = 12;
            int rc = pt_scene_load(b, scene, &o);
            if (rc == 0) {
                pt_scene_view v;
                if (pt_scene_builder_view(b, &v) == 0) {
                    // touch every node and leaf index the way the kernel's translation does
                    long long acc = 0;
                    for (int m = 0; m < v.mesh_num; m++) {
                        const pt_bvh_node_device* nodes = v.bvh_nodes[m];
                        for (int i = 0; i < nodes[0].next_node_index; i++) {
                            acc += nodes[i].next_node_index;
                            if (nodes[i].is_leaf && nodes[i].triangle_indices)
                                for (int k = 0; k < leaf; k++) acc += nodes[i].triangle_indices[k];
                        }
                    }
                    std::printf("scene %s method %d leaf %d: %d meshes, %d triangles (%lld)\n", scene, method, leaf,
                                v.mesh_num, v.triangle_num, acc);
                }
            } else {
                std::printf("scene %s method %d leaf %d: rc %d\n", scene, method, leaf, rc);
            }
            pt_scene_builder_destroy(b);
        }
    }
    return 0;
}

static int run_bvh(unsigned seed) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> u(-3.0f, 3.0f);
    pt_material mat;
    std::memset(&mat, 0, sizeof(mat));
    for (int n : {1, 2, 3, 7, 64, 1000}) {
        std::vector<pt_triangle> tris((size_t)n);
        for (auto& t : tris) {
            std::memset(&t, 0, sizeof(t));
            float* v = &t.vertex0.x;
            for (int k = 0; k < 9; k++) v[k] = (rng() % 5 == 0) ? 0.5f : u(rng);  // some coplanar / repeated values
            t.mat = &mat;
        }
        for (int method = 0; method < 2; method++)
            for (int leaf = 1; leaf <= 4; leaf++) {
                pt_bvh_node_device* nodes = nullptr;
                int nn = 0, ln = 0, *leafs = nullptr;
                int rc = pt_bvh_build_ex(tris.data(), n, 0, leaf, method, 12, &nodes, &nn, &leafs, &ln);
                if (rc == 0) pt_bvh_free(nodes, leafs);
            }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const char* mode = argv[1];
    if (!std::strcmp(mode, "config")) {
        for (int i = 2; i < argc; i++) {
            pt_configuration c;
            std::printf("config %s: %d\n", argv[i], pt_config_load(argv[i], &c));
        }
    } else if (!std::strcmp(mode, "obj")) {
        for (int i = 2; i < argc; i++) {
            pt_obj_mesh m;
            std::memset(&m, 0, sizeof(m));
            int rc = pt_obj_load(argv[i], &m);
            std::printf("obj %s: %d (%d triangles)\n", argv[i], rc, rc == 0 ? m.triangle_num : -1);
            if (rc == 0) pt_obj_free(&m);
        }
    } else if (!std::strcmp(mode, "image") && argc >= 3) {
        for (int i = 3; i < argc; i++) {
            int w = 0, h = 0;
            unsigned char* px = nullptr;
            int rc = pt_image_load(argv[i], &w, &h, &px);
            std::printf("image %s: %d (%dx%d)\n", argv[i], rc, w, h);
            if (rc == 0) {
                std::printf("  write: %d\n", pt_image_write_png(argv[2], w, h, px, 4));
                pt_image_free(px);
            }
        }
    } else if (!std::strcmp(mode, "scene") && argc >= 4) {
        return run_scene(argv[2], argv[3], argc > 5 ? argv[4] : nullptr, argc > 5 ? argv[5] : nullptr);
    } else if (!std::strcmp(mode, "bvh") && argc >= 3) {
        return run_bvh((unsigned)std::atoi(argv[2]));
    } else {
        return 2;
    }
    return 0;
}
