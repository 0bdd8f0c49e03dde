// capi.cpp — host half of the C ABI: errors, Tile::tile, scene generation.
#include <string.h>

#include <exception>
#include <string>

#include "../../include/rt.h"
#include "common.hpp"
#include "scene_builder.hpp"

namespace rthost {

static thread_local std::string g_error;

int set_error(int code, const std::string& msg) {
    g_error = msg;
    return code;
}
void clear_error() { g_error.clear(); }

}  // namespace rthost

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return rthost::g_error.c_str(); }

// Tile::tile, src/renderer.rs:242-296 (row-major, remainder column per row,
// then the remainder row, then the corner).
int rt_tile_image(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, rt_tile* out, uint32_t cap, uint32_t* count) {
    rthost::clear_error();
    if (tw == 0 || th == 0) return rthost::set_error(RT_ERR_INVALID, "tile size must be >= 1");
    if (!count) return rthost::set_error(RT_ERR_INVALID, "count is NULL");
    uint32_t nh = w / tw, rh = w % tw, nv = h / th, rv = h % th, n = 0;
    auto push = [&](uint32_t W, uint32_t H, uint32_t X, uint32_t Y) {
        if (out && n < cap) out[n] = rt_tile{W, H, X, Y};
        ++n;
    };
    for (uint32_t ty = 0; ty < nv; ++ty) {
        for (uint32_t tx = 0; tx < nh; ++tx) push(tw, th, tx * tw, ty * th);
        if (rh > 0) push(rh, th, nh * tw, ty * th);
    }
    if (rv > 0)
        for (uint32_t tx = 0; tx < nh; ++tx) push(tw, rv, tx * tw, nv * th);
    if (rh > 0 && rv > 0) push(rh, rv, nh * tw, nv * th);
    *count = n;
    return RT_OK;
}

int rt_scene_generate(const char* name, uint64_t seed, const char* asset_dir, rt_scene_desc** out) {
    rthost::clear_error();
    if (!name || !out) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    *out = nullptr;
    try {
        return rthost::generate_scene(name, seed, asset_dir ? asset_dir : ".", out);
    } catch (const std::bad_alloc&) {
        return rthost::set_error(RT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return rthost::set_error(RT_ERR_INVALID, e.what());
    }
}

void rt_scene_desc_free(rt_scene_desc* desc) {
    if (desc) rthost::SceneBuilder::free_desc(desc);
}

int rt_scene_background(const char* name, float rgb[3]) {
    rthost::clear_error();
    if (!name || !rgb) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    return rthost::scene_background(name, rgb);
}

}  // extern "C"
