// Graphics.cpp — the reference's static Graphics (Graphics.cpp:215-835) over the rmr C ABI.
// State lives in file-static globals as in the reference (Graphics.cpp:6-14, 215-261); the GPU
// objects (accumulator, scene tables, streams) are owned by the rmr context.
#include "Graphics.h"

#include <cstdio>
#include <iostream>

using Vector::Vector2;
using Vector::Vector3;

namespace {
Vector2 g_image_size(800, 600);  // Graphics.cpp:6
std::vector<std::string> g_materials, g_objects;
rmr_ctx* g_ctx = nullptr;
int g_device = 0;
std::vector<int> g_devices;       // setDevices: a device group instead of one context
rmr_group* g_group = nullptr;     // (g_ctx is then the first member's first context)
bool g_group_frame = false;       // SaveImage writes the group's last frame
int g_variant = RMR_VARIANT_RM3;  // Graphics.cpp:272 compiles RayMarch3
int g_status = RMR_OK;
std::string g_error;

bool check(int rc, const char* what) {
    g_status = rc;
    if (rc == RMR_OK) {
        g_error.clear();
        return true;
    }
    g_error = std::string(what) + ": " + (g_group ? rmr_group_last_error(g_group) : g_ctx ? rmr_last_error(g_ctx) : "no context");
    std::cerr << "Graphics::" << g_error << std::endl;  // the reference prints and continues
    return false;
}

bool need_ctx(const char* what) {
    if (g_ctx) return true;
    g_status = RMR_E_STATE;
    g_error = std::string(what) + ": Graphics::Init has not run";
    std::cerr << "Graphics::" << g_error << std::endl;
    return false;
}

std::string scene_json() {
    std::string s = "{\"materials\": [";
    for (size_t i = 0; i < g_materials.size(); i++) s += (i ? ", " : "") + g_materials[i];
    s += "], \"objects\": [";
    for (size_t i = 0; i < g_objects.size(); i++) s += (i ? ", " : "") + g_objects[i];
    return s + "]}";
}
}  // namespace

void Graphics::Init() {
    if (g_ctx) return;
    if (!g_devices.empty()) {
        const int rc = rmr_group_create(&g_group, g_devices.data(), (int)g_devices.size());
        if (rc != RMR_OK) {
            g_group = nullptr;
            g_status = rc;
            g_error = "Init: rmr_group_create failed (devices missing or RCCL unavailable)";
            std::cerr << "Graphics::" << g_error << std::endl;
            return;
        }
        g_ctx = rmr_group_context(g_group, 0, 0);
        Reload();
        return;
    }
    const int rc = rmr_create(&g_ctx, g_device);
    if (rc != RMR_OK) {
        g_ctx = nullptr;
        g_status = rc;
        g_error = "Init: no HIP device (rmr_create failed)";
        std::cerr << "Graphics::" << g_error << std::endl;
        return;
    }
    Reload();
}

void Graphics::Render(float currentTime, Vector2 min, Vector2 max, unsigned currentSample) {
    if (!need_ctx("Render")) return;
    check(rmr_render(g_ctx, currentTime, (float)min.x, (float)min.y, (float)max.x, (float)max.y, currentSample),
          "Render");
}

void Graphics::RenderSamples(const float* times, Vector2 min, Vector2 max, unsigned firstSample, unsigned nspp) {
    if (!need_ctx("RenderSamples")) return;
    check(rmr_render_spp(g_ctx, times, (int)min.x, (int)min.y, (int)max.x, (int)max.y, firstSample, nspp),
          "RenderSamples");
}

void Graphics::Reload() {
    if (!need_ctx("Reload")) return;
    int rc;
    if (g_group) {
        if (g_variant == RMR_VARIANT_RM3) {
            rc = rmr_group_load_builtin_scene(g_group, RMR_VARIANT_RM3);
        } else {
            const std::string js = scene_json();
            rc = rmr_group_load_scene_json(g_group, g_variant, js.c_str(), js.size());
        }
        if (!check(rc, "Reload(scene)")) return;
        if (!check(rmr_group_set_image_size(g_group, (int)g_image_size.x, (int)g_image_size.y), "Reload(size)")) return;
        check(rmr_group_reload(g_group), "Reload");
        g_group_frame = false;
        return;
    }
    if (g_variant == RMR_VARIANT_RM3) {
        rc = rmr_load_builtin_scene(g_ctx, RMR_VARIANT_RM3);  // RayMarch3's map is hard-coded
    } else {
        const std::string js = scene_json();
        rc = rmr_load_scene_json(g_ctx, g_variant, js.c_str(), js.size());
    }
    if (!check(rc, "Reload(scene)")) return;
    if (!check(rmr_set_image_size(g_ctx, (int)g_image_size.x, (int)g_image_size.y), "Reload(size)")) return;
    check(rmr_reload(g_ctx), "Reload");
}

void Graphics::SaveImage(std::string path) {
    if (!need_ctx("SaveImage")) return;
    if (g_group && g_group_frame) check(rmr_group_save_bmp(g_group, path.c_str()), "SaveImage");
    else check(rmr_save_bmp(g_ctx, path.c_str()), "SaveImage");
}

void Graphics::RenderFrame(const float* times, unsigned nspp) {
    if (!need_ctx("RenderFrame")) return;
    if (g_group) {
        if (check(rmr_group_render_frame(g_group, times, nspp), "RenderFrame")) g_group_frame = true;
        return;
    }
    check(rmr_render_spp(g_ctx, times, 0, 0, (int)g_image_size.x, (int)g_image_size.y, 0, nspp), "RenderFrame");
}

void Graphics::addMaterial(const std::string& materialJson) { g_materials.push_back(materialJson); }
void Graphics::addObject(const std::string& objectJson) { g_objects.push_back(objectJson); }
void Graphics::clearScene() {
    g_materials.clear();
    g_objects.clear();
}

void Graphics::setImageSize(Vector2 size) { g_image_size = size; }
Vector2 Graphics::getImageSize() { return g_image_size; }

void Graphics::setView(Vector3 eye, Vector3 ray00, Vector3 ray01, Vector3 ray10, Vector3 ray11) {
    if (!need_ctx("setView")) return;
    // glUniform3f takes floats (Graphics.cpp:830-834)
    const float e[3] = {(float)eye.x, (float)eye.y, (float)eye.z};
    const float a[3] = {(float)ray00.x, (float)ray00.y, (float)ray00.z};
    const float b[3] = {(float)ray01.x, (float)ray01.y, (float)ray01.z};
    const float c[3] = {(float)ray10.x, (float)ray10.y, (float)ray10.z};
    const float d[3] = {(float)ray11.x, (float)ray11.y, (float)ray11.z};
    if (g_group) check(rmr_group_set_view(g_group, e, a, b, c, d), "setView");
    else check(rmr_set_view(g_ctx, e, a, b, c, d), "setView");
}

void Graphics::setVariant(int variant) { g_variant = variant; }
int Graphics::getVariant() { return g_variant; }
void Graphics::setParams(const rmr_params& p) {
    if (!need_ctx("setParams")) return;
    if (g_group) check(rmr_group_set_params(g_group, &p), "setParams");
    else check(rmr_set_params(g_ctx, &p), "setParams");
}
rmr_params Graphics::getParams() {
    rmr_params p;
    rmr_default_params(&p);
    if (g_ctx) rmr_get_params(g_ctx, &p);
    return p;
}
void Graphics::setDevice(int device) { g_device = device; }
void Graphics::setDevices(const std::vector<int>& devices) { g_devices = devices; }
rmr_group* Graphics::group() { return g_group; }
void Graphics::setEnvMap(const unsigned char* rgba8, int w, int h) {
    if (!need_ctx("setEnvMap")) return;
    if (g_group) check(rmr_group_set_env_map(g_group, rgba8, w, h), "setEnvMap");
    else check(rmr_set_env_map(g_ctx, rgba8, w, h), "setEnvMap");
}
void Graphics::Sync() {
    if (!need_ctx("Sync")) return;
    if (g_group) check(rmr_group_sync(g_group), "Sync");
    else check(rmr_sync(g_ctx), "Sync");
}
bool Graphics::saveCheckpoint(const std::string& path, unsigned samplesDone) {
    return need_ctx("saveCheckpoint") && check(rmr_save_accum(g_ctx, path.c_str(), samplesDone), "saveCheckpoint");
}
bool Graphics::loadCheckpoint(const std::string& path, unsigned* samplesDone) {
    uint32_t n = 0;
    const bool ok = need_ctx("loadCheckpoint") && check(rmr_load_accum(g_ctx, path.c_str(), &n), "loadCheckpoint");
    if (ok && samplesDone) *samplesDone = n;
    return ok;
}
int Graphics::lastStatus() { return g_status; }
std::string Graphics::lastError() { return g_error; }
rmr_ctx* Graphics::context() { return g_ctx; }
void Graphics::Shutdown() {
    if (g_group) rmr_group_destroy(g_group);   // owns g_ctx
    else if (g_ctx) rmr_destroy(g_ctx);
    g_group = nullptr;
    g_ctx = nullptr;
}
