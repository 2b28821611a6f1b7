// Program.cpp — headless driver (rmr_cli): the reference's main loop (Program.cpp:86-323) and the
// console commands of CLI.cpp:190-218, without the SFML window / GUI.
//
//  * fixed-spp mode (samples > 0, Program.cpp:232-299): tiles of a gridW x gridH grid in the
//    outward spiral order of Program.cpp:113-115/203-222, each tile rendered to `samples` samples
//    before moving on;
//  * progressive mode (samples == 0, Program.cpp:184-231): every pass renders ONE sample of every
//    tile in spiral order, `--passes` passes;
//  * the seed uniform follows the deterministic schedule time(f, s) = 1000 f + 0.016 s (SURVEY
//    §8d) instead of the wall clock the reference passes (Program.cpp:319);
//  * by default a tile's samples go to the GPU in one batched call (Graphics::RenderSamples,
//    bitwise equal to the per-sample calls); --per-sample issues one Graphics::Render per sample
//    per tile exactly like the reference;
//  * save() writes output/<%Y-%m-%d_%H-%M-%S>.bmp (Program.cpp:71-84) unless --out is given;
//  * --gpus N / --devices a,b,..: the frame tile-partitioned over several GPUs of the node from this one
//    process (Graphics::setDevices -> librmr_group.so, one RCCL reduce per frame): the whole image
//    rendered as one frame of `samples` samples (or `passes` in progressive mode), bitwise the image
//    the tile loop gives wherever the grid covers it (every pixel gets the same seeds in the same order).
#include <sys/stat.h>
#include <dirent.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "Camera.h"
#include "Graphics.h"
#include "Screen.h"

using Vector::Vector2;
using Vector::Vector3;

namespace {

const float PI = 3.141592653f;  // Program.cpp:62

struct Options {
    std::string scene, out, checkpoint, resume, scene_dir = "scenes", env_map;
    int env_w = 0, env_h = 0;
    int variant = -1;
    int width = 800, height = 600;  // Graphics.cpp:6
    int samples = 128;              // Program.cpp:104
    int passes = 16;
    int grid_w = 4, grid_h = 4;     // Program.cpp:106-107
    int frame = 0;
    int device = 0;
    std::vector<int> devices;       // --gpus / --devices: the device group
    bool per_sample = false, interactive = false, quiet = false;
    bool print_tiles = false, print_view = false;  // host-only diagnostics (no GPU needed)
    rmr_params params;
    bool have_camera = false;
    double cam[6] = {0, 4, -6, 0, -3, 6};
};

// Program.cpp:113-115, 203-222: the outward spiral over the tile grid
std::vector<std::pair<int, int>> tile_spiral(int gw, int gh) {
    std::vector<std::pair<int, int>> order;
    int x = (int)std::ceil((float)gw / 2.0) - 1, y = (int)std::ceil((float)gh / 2.0) - 1;
    int dx = -1, dy = 0, passed = 0, last = 0, dist = 0;
    while (passed < gw * gh) {
        order.emplace_back(x, y);
        x -= gw / 2;
        y -= gh / 2;
        if (dist * 2 == passed - last) {
            dist++;
            last = passed;
            const int t = dx; dx = dy; dy = -t;
        } else if (dist == passed - last) {
            const int t = dx; dx = dy; dy = -t;
        }
        passed++;
        x += dx + gw / 2;
        y += dy + gh / 2;
    }
    return order;
}

float seed_time(int frame, unsigned s) { return (float)(1000.0 * frame + 0.016 * (double)s); }

std::string read_file(const std::string& path, bool* ok) {
    std::ifstream f(path, std::ios::binary);
    *ok = (bool)f;
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// Split a scene file's "materials" / "objects" arrays into per-element JSON texts for
// Graphics::addMaterial / addObject (CLI.cpp:63-75 addScene). A small bracket matcher: strings
// are skipped, so brackets inside names do not count.
bool split_array(const std::string& js, const std::string& key, std::vector<std::string>& out) {
    const size_t k = js.find("\"" + key + "\"");
    if (k == std::string::npos) return true;  // absent = empty
    size_t i = js.find('[', k);
    if (i == std::string::npos) return false;
    int depth = 0;
    size_t start = std::string::npos;
    bool in_str = false;
    for (; i < js.size(); i++) {
        const char c = js[i];
        if (in_str) {
            if (c == '\\') i++;
            else if (c == '"') in_str = false;
            continue;
        }
        if (c == '"') { in_str = true; continue; }
        if (c == '[' || c == '{') {
            if (depth == 1 && start == std::string::npos) start = i;
            depth++;
        } else if (c == ']' || c == '}') {
            depth--;
            if (depth == 1 && start != std::string::npos) {
                out.push_back(js.substr(start, i - start + 1));
                start = std::string::npos;
            }
            if (depth == 0) return true;
        }
    }
    return false;
}

bool load_scene(const std::string& path) {
    bool ok = false;
    const std::string js = read_file(path, &ok);
    if (!ok) {
        std::cout << "Failed to load file" << std::endl;  // CLI.cpp:58-61
        return false;
    }
    std::vector<std::string> mats, objs;
    if (!split_array(js, "materials", mats) || !split_array(js, "objects", objs)) {
        std::cout << "Failed to parse configuration" << std::endl;
        return false;
    }
    Graphics::clearScene();
    for (auto& m : mats) Graphics::addMaterial(m);
    for (auto& o : objs) Graphics::addObject(o);
    return true;
}

std::string save_name() {
    std::time_t t = std::time(nullptr);
    std::tm now;
    localtime_r(&t, &now);
    char buf[80];
    std::strftime(buf, sizeof buf, "%Y-%m-%d_%H-%M-%S", &now);
    return std::string(buf) + ".bmp";
}

void save(const Options& o) {  // Program.cpp:71-84
    std::string path = o.out;
    if (path.empty()) {
        mkdir("output", 0755);
        path = "output/" + save_name();
    }
    Graphics::SaveImage(path);
    if (Graphics::lastStatus() == RMR_OK) std::cout << "Saved image as: " << path << std::endl;
}

struct RenderResult {
    double seconds = 0;
    unsigned long long samples = 0;
};

// One render of the current scene: fixed-spp (samples > 0) or progressive (samples == 0).
RenderResult render(const Options& o, unsigned first_pass) {
    Graphics::Reload();
    Camera camera(Vector3(o.cam[0], o.cam[1], o.cam[2]), Vector3(o.cam[3], o.cam[4], o.cam[5]).normalized(),
                  (float)(Graphics::getImageSize().x / Graphics::getImageSize().y), PI / 4);
    if (!o.resume.empty()) {
        unsigned done = 0;
        if (Graphics::loadCheckpoint(o.resume, &done)) first_pass = done;
    }
    const int W = (int)Graphics::getImageSize().x, H = (int)Graphics::getImageSize().y;
    const int cw = W / o.grid_w, ch = H / o.grid_h;  // Program.cpp:108-109 (remainder not rendered)
    const auto order = tile_spiral(o.grid_w, o.grid_h);
    RenderResult r;
    Graphics::Sync();
    const auto t0 = std::chrono::steady_clock::now();
    auto tile_rect = [&](std::pair<int, int> t, Vector2& mn, Vector2& mx) {
        mn = Vector2(t.first * cw, t.second * ch);
        mx = Vector2((t.first + 1) * cw, (t.second + 1) * ch);
    };
    if (!o.devices.empty()) {   // the device group: one frame over the whole image
        const unsigned n = o.samples > 0 ? (unsigned)o.samples : (unsigned)o.passes;
        std::vector<float> times(n);
        for (unsigned s = 0; s < n; s++) times[s] = seed_time(o.frame, s);
        Graphics::RenderFrame(times.data(), n);
        if (Graphics::lastStatus() != RMR_OK) return r;
        Graphics::Sync();
        r.samples = (unsigned long long)n * (unsigned long long)W * H;
        r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return r;
    }
    if (o.samples > 0) {
        std::vector<float> times(o.samples);
        for (int s = 0; s < o.samples; s++) times[s] = seed_time(o.frame, s);
        for (auto t : order) {
            Vector2 mn, mx;
            tile_rect(t, mn, mx);
            if (o.per_sample) {
                for (int s = 0; s < o.samples; s++) Graphics::Render(times[s], mn, mx, (unsigned)s);
            } else {
                Graphics::RenderSamples(times.data(), mn, mx, 0, (unsigned)o.samples);
            }
            if (Graphics::lastStatus() != RMR_OK) return r;
        }
        r.samples = (unsigned long long)o.samples * (unsigned long long)cw * ch * order.size();
    } else {
        for (unsigned s = first_pass; s < first_pass + (unsigned)o.passes; s++) {
            const float tm = seed_time(o.frame, s);
            for (auto t : order) {
                Vector2 mn, mx;
                tile_rect(t, mn, mx);
                Graphics::Render(tm, mn, mx, s);
            }
            if (Graphics::lastStatus() != RMR_OK) return r;
            if (!o.quiet) std::cout << s << std::endl;  // Program.cpp:197
        }
        r.samples = (unsigned long long)o.passes * (unsigned long long)cw * ch * order.size();
        if (!o.checkpoint.empty()) Graphics::saveCheckpoint(o.checkpoint, first_pass + o.passes);
    }
    Graphics::Sync();
    r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (o.samples > 0 && !o.checkpoint.empty()) Graphics::saveCheckpoint(o.checkpoint, (unsigned)o.samples);
    return r;
}

void report(const Options& o, const RenderResult& r) {
    std::cout << "Render Time: " << r.seconds << std::endl;  // Program.cpp:297
    if (!o.quiet && r.seconds > 0)
        std::printf("{\"samples\": %llu, \"seconds\": %.6f, \"msamples_per_s\": %.3f}\n", r.samples, r.seconds,
                    r.samples / r.seconds / 1e6);
}

std::vector<std::string> list_scenes(const std::string& dir) {  // CLI.cpp:9-36 listNames
    std::vector<std::string> out;
    if (DIR* d = opendir(dir.c_str())) {
        while (dirent* e = readdir(d)) {
            std::string n = e->d_name;
            if (n.size() > 6 && n.find(".scene") != std::string::npos) out.push_back(dir + "/" + n);
        }
        closedir(d);
    }
    std::sort(out.begin(), out.end());
    return out;
}

bool read_int(int* dst) {
    std::string in;
    if (!(std::cin >> in)) return false;
    try {
        *dst = std::stoi(in);
    } catch (const std::exception&) {
        std::cout << "ERROR: Invalid Number" << std::endl;
    }
    return true;
}

// CLI.cpp:176-218: load_scene / samples / grid_width / grid_height / render / save (+ quit)
int interactive(Options o) {
    bool will_save = false;
    std::string cmd;
    while (std::cin >> cmd) {
        if (cmd == "load_scene") {
            const auto paths = list_scenes(o.scene_dir);
            for (size_t i = 0; i < paths.size(); i++)
                std::cout << "[" << i << "] " << paths[i].substr(paths[i].find_last_of('/') + 1) << std::endl;
            int idx = -1;
            if (!read_int(&idx)) break;
            if (idx < 0 || idx >= (int)paths.size()) {
                std::cout << "ERROR: Out of Range" << std::endl;
                continue;
            }
            load_scene(paths[idx]);
        } else if (cmd == "samples") {
            std::cout << "Enter number:" << std::endl;
            if (!read_int(&o.samples)) break;
        } else if (cmd == "grid_width") {
            std::cout << "Enter number:" << std::endl;
            if (!read_int(&o.grid_w)) break;
        } else if (cmd == "grid_height") {
            std::cout << "Enter number:" << std::endl;
            if (!read_int(&o.grid_h)) break;
        } else if (cmd == "render") {
            report(o, render(o, 0));
            if (will_save) {
                save(o);
                will_save = false;
            }
        } else if (cmd == "save") {
            will_save = true;
            if (Graphics::context()) {
                save(o);
                will_save = false;
            }
        } else if (cmd == "quit" || cmd == "exit") {
            break;
        } else {
            std::cout << "Unknown command: " << cmd << std::endl;
        }
    }
    return 0;
}

void usage() {
    std::puts(
        "rmr_cli — headless driver of the rmr SDF ray-march path tracer (Program.cpp / CLI.cpp)\n"
        "  --scene FILE        scene JSON (v1 format for rm1, v2 for rm2); none = RayMarch3 built-in\n"
        "  --variant rm1|rm2|rm3   (default rm1 with --scene, rm3 without)\n"
        "  --size WxH          image size (default 800x600)\n"
        "  --samples N         spp per tile (default 128); 0 = progressive\n"
        "  --passes P          progressive passes (default 16)\n"
        "  --grid GWxGH        tile grid (default 4x4)\n"
        "  --bounces B --max-steps N --max-dist D --step-mult S --separate-channels 0|1\n"
        "  --camera ex,ey,ez,dx,dy,dz   (default 0,4,-6,0,-3,6)\n"
        "  --env-map FILE WxH  raw RGBA8 envTex for skyColor (row 0 = up); enables useEnvTex\n"
        "  --frame F           seed schedule frame: time = 1000 F + 0.016 s\n"
        "  --per-sample        one Graphics::Render launch per sample per tile (reference pattern)\n"
        "  --out FILE.bmp      (default output/<timestamp>.bmp)\n"
        "  --checkpoint FILE   write the float accumulator at the end; --resume FILE continue from one\n"
        "  --device N  --interactive (CLI.cpp commands on stdin)  --scene-dir DIR  --quiet\n"
        "  --gpus N | --devices a,b,..  the frame tile-partitioned over those GPUs (one process, RCCL reduce)");
}

bool parse(int argc, char** argv, Options& o) {
    rmr_default_params(&o.params);
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&](const char* name) -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing value for %s\n", name);
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--scene") o.scene = next("--scene");
        else if (a == "--variant") {
            const std::string v = next("--variant");
            o.variant = v == "rm1" ? RMR_VARIANT_RM1 : v == "rm2" ? RMR_VARIANT_RM2 : v == "rm3" ? RMR_VARIANT_RM3 : -2;
            if (o.variant == -2) return false;
        } else if (a == "--size") {
            if (std::sscanf(next("--size"), "%dx%d", &o.width, &o.height) != 2) return false;
        } else if (a == "--samples") o.samples = std::atoi(next("--samples"));
        else if (a == "--passes") o.passes = std::atoi(next("--passes"));
        else if (a == "--grid") {
            if (std::sscanf(next("--grid"), "%dx%d", &o.grid_w, &o.grid_h) != 2) return false;
        } else if (a == "--bounces") o.params.max_bounces = std::atoi(next("--bounces"));
        else if (a == "--max-steps") o.params.max_steps = std::atoi(next("--max-steps"));
        else if (a == "--max-dist") o.params.max_dist = (float)std::atof(next("--max-dist"));
        else if (a == "--step-mult") o.params.step_multiply = (float)std::atof(next("--step-mult"));
        else if (a == "--separate-channels") o.params.separate_channels = std::atoi(next("--separate-channels"));
        else if (a == "--camera") {
            double* c = o.cam;
            if (std::sscanf(next("--camera"), "%lf,%lf,%lf,%lf,%lf,%lf", c, c + 1, c + 2, c + 3, c + 4, c + 5) != 6)
                return false;
            o.have_camera = true;
        } else if (a == "--frame") o.frame = std::atoi(next("--frame"));
        else if (a == "--per-sample") o.per_sample = true;
        else if (a == "--out") o.out = next("--out");
        else if (a == "--checkpoint") o.checkpoint = next("--checkpoint");
        else if (a == "--resume") o.resume = next("--resume");
        else if (a == "--device") o.device = std::atoi(next("--device"));
        else if (a == "--gpus") {
            const int n = std::atoi(next("--gpus"));
            if (n <= 0) return false;
            o.devices.clear();
            for (int d = 0; d < n; d++) o.devices.push_back(d);
        } else if (a == "--devices") {
            std::stringstream ss(next("--devices"));
            std::string item;
            o.devices.clear();
            while (std::getline(ss, item, ',')) o.devices.push_back(std::atoi(item.c_str()));
            if (o.devices.empty()) return false;
        }
        else if (a == "--interactive") o.interactive = true;
        else if (a == "--scene-dir") o.scene_dir = next("--scene-dir");
        else if (a == "--quiet") o.quiet = true;
        else if (a == "--env-map") {  // raw RGBA8 file + its size: skyColor's envTex, enables useEnvTex
            o.env_map = next("--env-map");
            if (std::sscanf(next("--env-map size"), "%dx%d", &o.env_w, &o.env_h) != 2) return false;
            o.params.use_env_tex = 1;
        }
        else if (a == "--print-tiles") o.print_tiles = true;
        else if (a == "--print-view") o.print_view = true;
        else if (a == "--help" || a == "-h") {
            usage();
            std::exit(0);
        } else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return false;
        }
    }
    if (o.variant < 0) o.variant = (o.scene.empty() && !o.interactive) ? RMR_VARIANT_RM3 : RMR_VARIANT_RM1;
    if (o.width <= 0 || o.height <= 0 || o.grid_w <= 0 || o.grid_h <= 0 || o.samples < 0 || o.passes < 0)
        return false;
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    if (!parse(argc, argv, o)) {
        usage();
        return 2;
    }
    if (o.print_tiles) {  // the spiral tile order, one "x y" per line
        for (auto t : tile_spiral(o.grid_w, o.grid_h)) std::printf("%d %d\n", t.first, t.second);
        return 0;
    }
    if (o.print_view) {  // Camera corner rays (camera names: ray00 ray10 ray01 ray11), %.9g
        Camera cam(Vector3(o.cam[0], o.cam[1], o.cam[2]), Vector3(o.cam[3], o.cam[4], o.cam[5]).normalized(),
                   (float)((double)o.width / (double)o.height), PI / 4);
        Vector3 r[4];
        cam.getRays(r[0], r[1], r[2], r[3]);
        for (auto& v : r) std::printf("%.9g %.9g %.9g\n", v.x, v.y, v.z);
        return 0;
    }
    Screen::setScreenSize(Vector2(1280, 720));  // Program.cpp:89
    Graphics::setDevice(o.device);
    if (!o.devices.empty()) {
        if (!o.checkpoint.empty() || !o.resume.empty() || o.interactive) {
            std::fprintf(stderr, "--gpus / --devices: no checkpoint, resume or interactive mode\n");
            return 2;
        }
        Graphics::setDevices(o.devices);
    }
    Graphics::setVariant(o.variant);
    Graphics::setImageSize(Vector2(o.width, o.height));
    if (!o.scene.empty() && !load_scene(o.scene)) return 1;
    Graphics::Init();
    if (!Graphics::context()) return 3;  // no device: fail loudly, there is no CPU path
    if (!o.interactive && Graphics::lastStatus() != RMR_OK) return 1;  // interactive: scene comes later
    Graphics::setParams(o.params);
    if (!o.env_map.empty()) {
        bool ok = false;
        const std::string tex = read_file(o.env_map, &ok);
        if (!ok || tex.size() != (size_t)o.env_w * o.env_h * 4) {
            std::cerr << "env map: cannot read " << o.env_w << "x" << o.env_h << " RGBA8 from " << o.env_map << std::endl;
            return 1;
        }
        Graphics::setEnvMap((const unsigned char*)tex.data(), o.env_w, o.env_h);
    }
    if (o.interactive) return interactive(o);
    const RenderResult r = render(o, 0);
    if (Graphics::lastStatus() != RMR_OK) return 1;
    report(o, r);
    save(o);
    const int rc = Graphics::lastStatus() == RMR_OK ? 0 : 1;
    Graphics::Shutdown();
    return rc;
}
