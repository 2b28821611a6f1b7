// rmr_display.hip — Graphics::Display (Graphics.cpp:356-390) headless: the accumulator drawn as the
// reference's textured screen quad (createFQ, Graphics.cpp:227-258; FullQuad.vs / FullQuad.fs) into
// an RGBA8 screen image, with GL_FRAMEBUFFER_SRGB's linear -> sRGB encode and the SRC_ALPHA /
// ONE_MINUS_SRC_ALPHA blend (Graphics.cpp:268-269) of the fragment's alpha 1 / 0.
//
// One thread per screen pixel (row 0 = top: FullQuad.vs flips y). Per pixel, in float:
//   quad   x in [c - h, c + h), rows y in (c - h, c + h] (GL's edge rule with FullQuad.vs's y flip),
//          h = (imageSize / 2) * zoom; fragment centre pos = pixel + 0.5
//   uv     (pos - (c - h)) / ((c + h) - (c - h));  texel = floor(uv * imageSize) mod imageSize
//          (GL_NEAREST, Graphics.h:90-91, and GL_REPEAT, the default wrap; row 0 of the texture =
//          accumulator row 0)
//   colour texel.rgb, alpha 1 where min <= pos <= max (FullQuad.fs bounds test), else alpha 0
//   blend  alpha 1: the sRGB-encoded colour replaces the pixel; alpha 0 and pixels outside the
//          quad keep the caller's background
//   sRGB   byte = round(255 * srgb(clamp(c, 0, 1))) exactly: the 255 decision points of that
//          function in linear space (host, double, rounded up to float) bracket c; NaN -> 0.
// HBM-bound: 4 B read-modify-write per screen pixel plus one 16-B texel read (L2-resident reuse
// when zoom > 1).
#include <hip/hip_runtime.h>

#include "rmr_internal.h"

namespace rmr {

struct DisplayParams {
    const float4* accum;
    int img_w, img_h;
    float cx, cy, zoom;
    float min_x, min_y, max_x, max_y;
    int scr_w, scr_h;
    uint32_t* rgba8;            // screen image, RGBA8 little-endian words, row 0 = top
    const float* thr;           // [256]: thr[k] = smallest float c with byte(c) >= k (k >= 1); thr[0] = 0
};

__device__ __forceinline__ uint32_t srgb_byte(const float* __restrict__ thr, float c) {
    if (!(c > 0.0f)) return 0u;    // <= 0 and NaN
    if (c >= thr[255]) return 255u;
    // the approximate inverse (bare v_log / v_exp) lands within one of the answer; the bracket
    // thr[v] <= c < thr[v + 1] then fixes it
    const float s = (c < 0.0031308f) ? 12.92f * c : 1.055f * __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(c) * (1.0f / 2.4f)) - 0.055f;
    int v = (int)(s * 255.0f + 0.5f);
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    if (c < thr[v]) {
        do { v--; } while (v > 0 && c < thr[v]);
    } else {
        while (v < 255 && c >= thr[v + 1]) v++;
    }
    return (uint32_t)v;
}

__global__ __launch_bounds__(256) void k_display(DisplayParams D) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= D.scr_w || y >= D.scr_h) return;
    const float hw = ((float)D.img_w / 2.0f) * D.zoom, hh = ((float)D.img_h / 2.0f) * D.zoom;
    const float x0 = D.cx - hw, x1 = D.cx + hw, y0 = D.cy - hh, y1 = D.cy + hh;
    const float px = (float)x + 0.5f, py = (float)y + 0.5f;
    // rasterized: GL's tie rule for a lower-left window origin (left and bottom edges in, in window
    // coordinates; FullQuad.vs flips y, so in screen rows the quad is (y0, y1])
    if (!(px >= x0 && px < x1 && py > y0 && py <= y1)) return;
    if (!(px >= D.min_x && px <= D.max_x && py >= D.min_y && py <= D.max_y)) return;  // alpha 0
    const float u = (px - x0) / (x1 - x0), v = (py - y0) / (y1 - y0);
    // GL_REPEAT (the texture's default wrap: Framebuffer::Create sets only the filters), so the
    // quad's included bottom row (v = 1) samples texel row 0, as the reference draws it
    int i = (int)floorf(u * (float)D.img_w) % D.img_w, j = (int)floorf(v * (float)D.img_h) % D.img_h;
    i += i < 0 ? D.img_w : 0;
    j += j < 0 ? D.img_h : 0;
    const float4 t = D.accum[(size_t)j * D.img_w + i];
    const uint32_t r = srgb_byte(D.thr, t.x), g = srgb_byte(D.thr, t.y), b = srgb_byte(D.thr, t.z);
    D.rgba8[(size_t)y * D.scr_w + x] = r | (g << 8) | (b << 16) | (255u << 24);
}

hipError_t launch_display(const float4* accum, int img_w, int img_h, float cx, float cy, float zoom, float min_x,
                          float min_y, float max_x, float max_y, int scr_w, int scr_h, uint32_t* rgba8,
                          const float* thr, hipStream_t s) {
    DisplayParams D{accum, img_w, img_h, cx, cy, zoom, min_x, min_y, max_x, max_y, scr_w, scr_h, rgba8, thr};
    dim3 grid((unsigned)((scr_w + 63) / 64), (unsigned)((scr_h + 3) / 4));
    k_display<<<grid, 256, 0, s>>>(D);
    return hipGetLastError();
}

}  // namespace rmr
