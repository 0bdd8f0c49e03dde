// shimmer_cli.cpp — command-line drop-in for the reference binary (src/main.rs:35-183).
//
// Same positional scene names and flags as the clap `Cli` (src/main.rs:51-103),
// same background table (:155-164), same image height rule
// (H = (W as f32 / aspect) as usize, src/renderer.rs:34-39) and the same ASCII
// P3 PPM on stdout (src/renderer.rs:107-127). The render itself runs on the
// GPU through the C ABI, and so does the output step: the image never leaves
// the device as floats, rt_format_ppm quantises and formats the P3 body there.
// There is no CPU fallback.
//
// Extra flags (not in the reference): --seed N (the reference's thread_rng is
// OS-seeded), --assets DIR, --device N, --devices N (one frame over devices
// 0..N-1, rt_render_multi), --pfm FILE (linear float dump), --exact-bvh, --hrpp.
//
// HRPP: the reference CLI renders showcase, bunny, gargoyle and igea-hrpp with
// hash-based ray path predictors on (Bvh::with_predictor, src/main.rs:586, 679,
// 685, 828), i.e. with an approximate, non-deterministic traversal. This CLI
// renders exactly by default (the bit-reproducible path); --hrpp turns on the
// GPU HRPP experiment (RT_FLAG_HRPP) for the BVHs those scenes build with a
// predictor, which approximates the reference's default output. Parity with the
// reference's HRPP images cannot be pinned: they depend on thread timing.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/rt.h"

namespace {

void usage() {
    fprintf(stderr,
            "Usage: shimmer <SCENE> [OPTIONS]\n"
            "  SCENE: random-spheres random-moving-spheres two-spheres marble earth simple-lights\n"
            "         cornell cornell-smoke showcase bunny gargoyle igea-hrpp\n"
            "  -w, --image-width <W>            [default: 1080]\n"
            "  -a, --aspect-ratio <X> <Y>       [default: 16 9]\n"
            "  -s, --samples-per-pixel <N>      [default: 500]\n"
            "  -d, --depth <N>                  [default: 50]\n"
            "      --tile-width <N>             [default: 8]\n"
            "      --tile-height <N>            [default: 8]\n"
            "      --cam-look-from <X> <Y> <Z>  [default: 13 2 3]\n"
            "      --cam-look-at <X> <Y> <Z>    [default: 0 0 0]\n"
            "      --cam-view-up <X> <Y> <Z>    [default: 0 1 0]\n"
            "      --cam-vertical-fov <DEG>     [default: 20]\n"
            "      --cam-aperture <A>           [default: 0]\n"
            "      --cam-focus-dist <D>         [default: 10]\n"
            "      --cam-start-time <T>         [default: 0]\n"
            "      --cam-end-time <T>           [default: 0]\n"
            "      --seed <N> --assets <DIR> --device <N> --devices <N> --pfm <FILE> --exact-bvh\n"
            "      --hrpp   hash-based ray path prediction on the scene's predictor BVHs (approximate;\n"
            "               the reference's default for showcase / bunny / gargoyle / igea-hrpp)\n");
}

bool parse_f(const char* s, float* out) {
    char* end = nullptr;
    *out = strtof(s, &end);
    return end && *end == '\0';
}
bool parse_u(const char* s, unsigned long long* out) {
    char* end = nullptr;
    *out = strtoull(s, &end, 10);
    return end && *end == '\0';
}

std::string default_assets(const char* argv0) {
    std::string p(argv0);
    size_t k = p.rfind('/');
    std::string dir = k == std::string::npos ? "." : p.substr(0, k);
    return dir + "/../../assets";
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        usage();
        return 2;
    }
    std::string scene;
    unsigned long long width = 1080, spp = 500, depth = 50, tw = 8, th = 8, seed = 1, device = 0, devices = 1;
    float aspect[2] = {16.0f, 9.0f};
    float from[3] = {13.0f, 2.0f, 3.0f}, at[3] = {0.0f, 0.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
    float vfov = 20.0f, aperture = 0.0f, focus = 10.0f, t0 = 0.0f, t1 = 0.0f;
    std::string assets = default_assets(argv[0]), pfm;
    bool exact = false, hrpp = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto need = [&](int n) {
            if (i + n >= argc) {
                fprintf(stderr, "error: %s needs %d value(s)\n", a.c_str(), n);
                exit(2);
            }
        };
        auto fl = [&](float* dst, int n) {
            need(n);
            for (int k = 0; k < n; ++k)
                if (!parse_f(argv[++i], &dst[k])) {
                    fprintf(stderr, "error: bad number for %s\n", a.c_str());
                    exit(2);
                }
        };
        auto ul = [&](unsigned long long* dst) {
            need(1);
            if (!parse_u(argv[++i], dst)) {
                fprintf(stderr, "error: bad integer for %s\n", a.c_str());
                exit(2);
            }
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "-w" || a == "--image-width") ul(&width);
        else if (a == "-a" || a == "--aspect-ratio") fl(aspect, 2);
        else if (a == "-s" || a == "--samples-per-pixel") ul(&spp);
        else if (a == "-d" || a == "--depth") ul(&depth);
        else if (a == "--tile-width") ul(&tw);
        else if (a == "--tile-height") ul(&th);
        else if (a == "--cam-look-from") fl(from, 3);
        else if (a == "--cam-look-at") fl(at, 3);
        else if (a == "--cam-view-up") fl(up, 3);
        else if (a == "--cam-vertical-fov") fl(&vfov, 1);
        else if (a == "--cam-aperture") fl(&aperture, 1);
        else if (a == "--cam-focus-dist") fl(&focus, 1);
        else if (a == "--cam-start-time") fl(&t0, 1);
        else if (a == "--cam-end-time") fl(&t1, 1);
        else if (a == "--seed") ul(&seed);
        else if (a == "--device") ul(&device);
        else if (a == "--devices") ul(&devices);
        else if (a == "--assets") { need(1); assets = argv[++i]; }
        else if (a == "--pfm") { need(1); pfm = argv[++i]; }
        else if (a == "--exact-bvh") exact = true;
        else if (a == "--hrpp") hrpp = true;
        else if (!a.empty() && a[0] == '-') { fprintf(stderr, "error: unexpected argument '%s'\n", a.c_str()); usage(); return 2; }
        else if (scene.empty()) scene = a;
        else { fprintf(stderr, "error: unexpected argument '%s'\n", a.c_str()); return 2; }
    }
    if (scene.empty()) { usage(); return 2; }
    float aspect_ratio = aspect[0] / aspect[1];                                   // main.rs:109
    unsigned long long height = (unsigned long long)((float)width / aspect_ratio);  // renderer.rs:37

    rt_camera_desc cam;
    memset(&cam, 0, sizeof cam);
    memcpy(cam.look_from, from, sizeof from);
    memcpy(cam.look_at, at, sizeof at);
    memcpy(cam.view_up, up, sizeof up);
    cam.vfov_deg = vfov;
    cam.aspect_ratio = aspect_ratio;
    cam.aperture = aperture;
    cam.focus_dist = focus;
    cam.time0 = t0;
    cam.time1 = t1;

    auto start = std::chrono::steady_clock::now();  // main.rs:138
    rt_scene_desc* desc = nullptr;
    if (rt_scene_generate(scene.c_str(), seed, assets.c_str(), &desc) != RT_OK) {
        fprintf(stderr, "error: %s\n", rt_last_error());
        return 1;
    }
    rt_render_params p;
    memset(&p, 0, sizeof p);
    p.width = (uint32_t)width;
    p.height = (uint32_t)height;
    p.samples_per_pixel = (uint32_t)spp;
    p.max_depth = (uint32_t)depth;
    p.tile_width = (uint32_t)tw;
    p.tile_height = (uint32_t)th;
    p.seed = seed;
    p.flags = (exact ? RT_FLAG_EXACT_BVH : 0u) | (hrpp ? RT_FLAG_HRPP : 0u);
    if (rt_scene_background(scene.c_str(), p.background) != RT_OK) {
        fprintf(stderr, "error: %s\n", rt_last_error());
        return 1;
    }
    const unsigned long long ndev = devices < 1 ? 1 : devices;
    std::vector<rt_scene_handle> handles(ndev, nullptr);
    auto fail = [&](const char* what) {
        fprintf(stderr, "error: %s: %s\n", what, rt_last_error());
        for (rt_scene_handle x : handles)
            if (x) rt_scene_free(x);
        rt_scene_desc_free(desc);
        return 1;
    };
    for (unsigned long long i = 0; i < ndev; ++i)
        if (rt_scene_upload(desc, (int)(ndev > 1 ? i : device), &handles[i]) != RT_OK) return fail("rt_scene_upload");
    const int dev0 = (int)(ndev > 1 ? 0 : device);
    const size_t npix = (size_t)width * height, fbytes = npix * 3u * sizeof(float);
    float* d_out = nullptr;
    char* d_text = nullptr;
    unsigned long long* d_seg = nullptr;
    hipStream_t st = nullptr;
    if (hipSetDevice(dev0) != hipSuccess || hipStreamCreate(&st) != hipSuccess || hipMalloc(&d_out, fbytes) != hipSuccess ||
        hipMalloc(&d_seg, sizeof *d_seg) != hipSuccess || hipMalloc(&d_text, npix * 12u + 1u) != hipSuccess ||
        hipMemsetAsync(d_out, 0, fbytes, st) != hipSuccess || hipMemsetAsync(d_seg, 0, sizeof *d_seg, st) != hipSuccess) {
        fprintf(stderr, "error: device allocation failed\n");
        return 1;
    }
    rt_stats st_multi;
    memset(&st_multi, 0, sizeof st_multi);
    std::vector<float> img;
    fprintf(stderr, "Rendering tiles...\n");
    if (ndev > 1) {  // one frame over several devices, gathered on the host, then back to device 0
        img.assign(npix * 3u, 0.0f);
        if (rt_render_multi(handles.data(), (uint32_t)ndev, &cam, &p, img.data(), &st_multi) != RT_OK)
            return fail("rt_render_multi");
        if (hipMemcpyAsync(d_out, img.data(), fbytes, hipMemcpyHostToDevice, st) != hipSuccess) return fail("H2D");
    } else if (rt_render_launch(handles[0], &cam, &p, d_out, d_seg, st) != RT_OK) {
        return fail("rt_render_launch");
    }
    fprintf(stderr, "\nDone tracing.\nWriting to file...\n");
    uint64_t text_bytes = 0;
    if (rt_format_ppm(d_out, (uint32_t)width, (uint32_t)height, d_text, npix * 12u + 1u, &text_bytes, st) != RT_OK)
        return fail("rt_format_ppm");
    std::string out;
    char line[64];
    snprintf(line, sizeof line, "P3\n%llu %llu\n255\n", width, height);
    out = line;
    const size_t head = out.size();
    out.resize(head + text_bytes);
    unsigned long long seg = 0;
    if (hipMemcpy(&out[head], d_text, text_bytes, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&seg, d_seg, sizeof seg, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("D2H");
    fwrite(out.data(), 1, out.size(), stdout);
    fflush(stdout);
    fprintf(stderr, "Done writing to file.\n");
    if (!pfm.empty()) {
        if (img.empty()) {
            img.resize(npix * 3u);
            (void)hipMemcpy(img.data(), d_out, fbytes, hipMemcpyDeviceToHost);
        }
        FILE* f = fopen(pfm.c_str(), "wb");
        if (f) {
            fprintf(f, "PF\n%llu %llu\n-1.0\n", width, height);  // PFM rows are bottom-up, like ours
            fwrite(img.data(), sizeof(float), img.size(), f);
            fclose(f);
        }
    }
    (void)hipFree(d_out);
    (void)hipFree(d_text);
    (void)hipFree(d_seg);
    (void)hipStreamDestroy(st);
    for (rt_scene_handle x : handles) rt_scene_free(x);
    rt_scene_desc_free(desc);
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    fprintf(stderr, "Render time: %.3fs (%llu devices, %llu segments)\n", secs, ndev,
            ndev > 1 ? (unsigned long long)st_multi.segments : seg);
    return 0;
}
