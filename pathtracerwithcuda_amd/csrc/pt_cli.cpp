// pt_cli.cpp — pt_render, the headless host program around the render call.
//
// It does what the reference application does between start-up and a screenshot, without the
// window (Main/window.cpp:115-225 init_all, :381-412 render, :712-740 screenshot):
//   config_parser::load_config          -> pt_config_load           (res/configuration/config.json)
//   scene_parser::load_scene + create_scene_data_device -> pt_scene_load (JSON, OBJ, images, BVH)
//   view_camera (orbit camera) -> render_camera          -> pt_view_camera_*  (Core/camera.cpp)
//   path_tracer::render, pass after pass                 -> path_tracer_kernel (--abi) or the
//                                                          resident native API (default)
//   screenshot                                           -> pt_image_write_png (+ optional PFM)
// and prints one JSON line with the timing (the reference shows FPS / frame time in its UI panel,
// Main/window.cpp:442-481).
//
//   pt_render --scene res/scene/cornell_box_simple.json --root <gpu_path_tracer dir>
//             [--config config.json] [--width W --height H] [--spp N] [--depth D]
//             [--yaw Y --pitch P --radius R --center x,y,z --aperture A --focal F --fov DEG]
//             [--background DIR --background-format FMT] [--abi] [--device N]
//             [--out image.png] [--pfm image.pfm]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/path_tracer_kernel.h"
#include "../../include/pt_host.h"
#include "../../include/pt_loader.h"
#include "../../include/pt_native.h"

namespace {

struct Args {
    std::string scene, root, config, background, background_format, out, pfm;
    int width = 0, height = 0, spp = 8, depth = -1, device = 0;
    float yaw = 0.0f, pitch = 0.3f, radius = 14.0f, aperture = 0.0f, focal = -1.0f, fov = 45.0f;
    float center[3] = {0.0f, 0.0f, 0.0f};
    bool abi = false;
};

void usage() {
    std::fprintf(stderr,
                 "usage: pt_render --scene FILE [--root DIR] [--config FILE] [--width W] [--height H] [--spp N]\n"
                 "                 [--depth D] [--yaw Y] [--pitch P] [--radius R] [--center x,y,z] [--aperture A]\n"
                 "                 [--focal F] [--fov DEG] [--background DIR] [--background-format FMT] [--abi]\n"
                 "                 [--device N] [--out FILE.png] [--pfm FILE.pfm]\n");
}

bool parse(int argc, char** argv, Args& a) {
    for (int i = 1; i < argc; i++) {
        std::string k = argv[i];
        auto val = [&](void) -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "[Error]missing value for %s\n", k.c_str()); return nullptr; }
            return argv[++i];
        };
        const char* v = nullptr;
        if (k == "--abi") { a.abi = true; continue; }
        if (k == "--help" || k == "-h") return false;
        if (!(v = val())) return false;
        if (k == "--scene") a.scene = v;
        else if (k == "--root") a.root = v;
        else if (k == "--config") a.config = v;
        else if (k == "--background") a.background = v;
        else if (k == "--background-format") a.background_format = v;
        else if (k == "--out") a.out = v;
        else if (k == "--pfm") a.pfm = v;
        else if (k == "--width") a.width = std::atoi(v);
        else if (k == "--height") a.height = std::atoi(v);
        else if (k == "--spp") a.spp = std::atoi(v);
        else if (k == "--depth") a.depth = std::atoi(v);
        else if (k == "--device") a.device = std::atoi(v);
        else if (k == "--yaw") a.yaw = std::strtof(v, nullptr);
        else if (k == "--pitch") a.pitch = std::strtof(v, nullptr);
        else if (k == "--radius") a.radius = std::strtof(v, nullptr);
        else if (k == "--aperture") a.aperture = std::strtof(v, nullptr);
        else if (k == "--focal") a.focal = std::strtof(v, nullptr);
        else if (k == "--fov") a.fov = std::strtof(v, nullptr);
        else if (k == "--center") {
            if (std::sscanf(v, "%f,%f,%f", &a.center[0], &a.center[1], &a.center[2]) != 3) return false;
        } else {
            std::fprintf(stderr, "[Error]unknown option %s\n", k.c_str());
            return false;
        }
    }
    return !a.scene.empty();
}

int write_pfm(const char* path, int w, int h, const std::vector<pt_float3>& img, int passes) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return -1;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", w, h);
    std::vector<float> row((size_t)w * 3);
    for (int y = h - 1; y >= 0; y--) {  // PFM rows run bottom to top; the running sum / passes = the mean
        for (int x = 0; x < w; x++) {
            const pt_float3& p = img[(size_t)y * w + x];
            row[(size_t)x * 3 + 0] = p.x / (float)passes;
            row[(size_t)x * 3 + 1] = p.y / (float)passes;
            row[(size_t)x * 3 + 2] = p.z / (float)passes;
        }
        std::fwrite(row.data(), sizeof(float), row.size(), f);
    }
    std::fclose(f);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    Args a;
    if (!parse(argc, argv, a)) { usage(); return 2; }

    pt_configuration cfg;
    if (!a.config.empty()) {
        if (pt_config_load(a.config.c_str(), &cfg) != 0) return 3;
    } else {
        pt_configuration_default(&cfg);
    }
    if (a.width > 0) cfg.width = a.width;
    if (a.height > 0) cfg.height = a.height;
    if (a.depth >= 0) cfg.max_tracer_depth = a.depth;
    const int W = cfg.width, H = cfg.height, P = W * H;
    if (W <= 0 || H <= 0 || a.spp <= 0) { std::fprintf(stderr, "[Error]empty frame\n"); return 2; }

    pt_scene_builder* b = pt_scene_builder_create();
    pt_scene_load_options opt;
    std::memset(&opt, 0, sizeof(opt));
    opt.root_dir = a.root.empty() ? nullptr : a.root.c_str();
    opt.background_override = a.background.empty() ? nullptr : a.background.c_str();
    opt.background_format = a.background_format.empty() ? nullptr : a.background_format.c_str();
    opt.leaf_size = cfg.bvh_leaf_node_triangle_num;
    opt.bvh_method = cfg.bvh_build;
    opt.bucket_num = cfg.bvh_bucket_max_divide_internal_num;
    const auto t_load = std::chrono::steady_clock::now();
    if (pt_scene_load(b, a.scene.c_str(), &opt) != 0) { pt_scene_builder_destroy(b); return 4; }
    pt_scene_view v;
    pt_scene_builder_view(b, &v);
    const double load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_load).count();

    // init_camera (Main/window.cpp:356-360) with the orbit parameters of the command line
    pt_view_camera vc;
    pt_view_camera_default(&vc);
    vc.center = {a.center[0], a.center[1], a.center[2]};
    vc.yaw = a.yaw; vc.pitch = a.pitch; vc.radius = a.radius;
    vc.aperture_radius = a.aperture;
    vc.focal_distance = a.focal > 0.0f ? a.focal : a.radius;
    pt_view_camera_set_resolution(&vc, (float)W, (float)H);
    pt_view_camera_set_fov(&vc, a.fov);
    pt_render_camera cam;
    pt_view_camera_get_render_camera(&vc, &cam);

    std::vector<pt_float3> img((size_t)P);
    std::vector<pt_uchar3> img8((size_t)P);
    double render_ms = 0.0;
    unsigned long long segments = 0;
    int rc = 0;
    if (a.abi) {
        // path_tracer::render (Core/path_tracer.cpp:40-67): pass_counter++, one call per pass
        void *s0 = nullptr, *s1 = nullptr, *s2 = nullptr, *s3 = nullptr, *s4 = nullptr;
        path_tracer_kernel_memory_allocate((pt_float3**)&s0, (pt_float3**)&s1, (pt_ray**)&s2, (int**)&s3,
                                           (pt_scattering**)&s4, P);
        const auto t0 = std::chrono::steady_clock::now();
        for (int pass = 1; pass <= a.spp; pass++)
            path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, P, img.data(), img8.data(),
                               pass, &cam, v.sky_cube_map, (pt_float3*)s0, (pt_float3*)s1, (pt_ray*)s2, (int*)s3,
                               (pt_scattering*)s4, v.mesh_textures, &cfg);
        render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        path_tracer_kernel_memory_free((pt_float3*)s0, (pt_float3*)s1, (pt_ray*)s2, (int*)s3, (pt_scattering*)s4);
        if (pt_last_error() && *pt_last_error()) rc = 5;
    } else {
        pt_context* ctx = nullptr;
        if (pt_context_create(a.device, &ctx) != PT_OK) {
            std::fprintf(stderr, "[Error]%s\n", pt_last_error());
            pt_scene_builder_destroy(b);
            return 5;
        }
        rc = pt_scene_upload(ctx, v.mesh_num, v.bvh_nodes, v.triangles, v.triangle_num, v.sphere_num, v.spheres,
                             v.sky_cube_map, v.mesh_textures, v.texture_num, &cfg);
        if (rc == PT_OK) rc = pt_frame_setup(ctx, W, H, nullptr);
        if (rc == PT_OK) rc = pt_stats_reset(ctx);
        if (rc == PT_OK) rc = pt_synchronize(ctx);
        const auto t0 = std::chrono::steady_clock::now();
        if (rc == PT_OK) rc = pt_render_passes(ctx, &cam, &cfg, 1, a.spp, 2);
        if (rc == PT_OK) rc = pt_synchronize(ctx);
        render_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        unsigned long long nodes = 0, tris = 0;
        if (rc == PT_OK) rc = pt_stats(ctx, &segments, &nodes, &tris);
        if (rc == PT_OK) rc = pt_image_download(ctx, img.data(), img8.data());
        if (rc != PT_OK) std::fprintf(stderr, "[Error]%s\n", pt_last_error());
        pt_context_destroy(ctx);
        rc = rc == PT_OK ? 0 : 5;
    }
    if (rc == 0 && !a.out.empty() && pt_image_write_png(a.out.c_str(), W, H, &img8[0].x, 3) != 0) rc = 6;
    if (rc == 0 && !a.pfm.empty() && write_pfm(a.pfm.c_str(), W, H, img, a.spp) != 0) rc = 6;
    std::printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"max_depth\": %d, \"path\": \"%s\", "
                "\"triangles\": %d, \"spheres\": %d, \"load_ms\": %.3f, \"render_ms\": %.3f, \"ms_per_pass\": %.4f, "
                "\"segments\": %llu, \"mrays_per_s\": %.3f, \"rc\": %d}\n",
                a.scene.c_str(), W, H, a.spp, cfg.max_tracer_depth, a.abi ? "reference-abi" : "native", v.triangle_num,
                v.sphere_num, load_ms, render_ms, render_ms / a.spp, segments,
                render_ms > 0 ? (double)segments / (render_ms * 1e3) : 0.0, rc);
    pt_scene_builder_destroy(b);
    return rc;
}
