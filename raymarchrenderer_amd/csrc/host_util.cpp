// host_util.cpp — host-side pieces of the drop-in boundary that need no GPU:
//   * rmr_camera_view: Camera::calculateRays (Camera.cpp:25-102) + the setView argument swap
//     (Camera.cpp:101 -> Graphics.cpp:827-835);
//   * rmr_encode_bmp: Graphics::SaveImage's output encoding (Graphics.cpp:754-799) and the BMP
//     writer of SOIL's stb_image_write (24-bit, BGR, bottom-up, alpha composited on (255,0,255)).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../../include/rmr.h"

namespace {

// Vector3::cross (double), Vector.h:327-330
void cross_d(const double a[3], const double b[3], double out[3]) {
    out[0] = a[1] * b[2] - a[2] * b[1];
    out[1] = a[2] * b[0] - a[0] * b[2];
    out[2] = a[0] * b[1] - a[1] * b[0];
}

// rotAxis(u, t, point, origin = 0), Camera.cpp:31-52. glm::mat3(a..i) is column-major, so
// uc's columns are (0,-uz,uy), (uz,0,-ux), (-uy,ux,0). Float arithmetic as in glm.
void rot_axis(const double u[3], float t, const double point[3], double out[3]) {
    const float ux = (float)u[0], uy = (float)u[1], uz = (float)u[2];
    const float uc[3][3] = {{0.0f, -uz, uy}, {uz, 0.0f, -ux}, {-uy, ux, 0.0f}};
    const float ut[3][3] = {{(float)(u[0] * u[0]), (float)(u[0] * u[1]), (float)(u[0] * u[2])},
                            {(float)(u[0] * u[1]), (float)(u[1] * u[1]), (float)(u[1] * u[2])},
                            {(float)(u[0] * u[2]), (float)(u[1] * u[2]), (float)(u[2] * u[2])}};
    const float c = std::cos(t), s = std::sin(t), omc = 1.0f - c;
    float R[3][3];
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) {
            const float id = (i == j) ? 1.0f : 0.0f;
            R[j][i] = (c * id + s * uc[j][i]) + omc * ut[j][i];
        }
    const float v[3] = {(float)point[0], (float)point[1], (float)point[2]};
    for (int i = 0; i < 3; i++) {
        const float p = R[0][i] * v[0] + R[1][i] * v[1] + R[2][i] * v[2];
        out[i] = (double)p;
    }
}

}  // namespace

extern "C" void rmr_camera_view(const double eye[3], const double dir[3], float aspect, float fov,
                                float out_eye[3], float out_ray00[3], float out_ray01[3],
                                float out_ray10[3], float out_ray11[3]) {
    const float v_angle = fov;
    const float h_angle = 2.0f * std::atan(aspect * std::tan(v_angle / 2.0f));
    const double up[3] = {0.0, 1.0, 0.0};
    double x[3], y[3];
    cross_d(dir, up, x);  // getLocal, Camera.cpp:25-29
    cross_d(dir, x, y);
    double r00[3], r10[3], r01[3], r11[3], tmp[3];
    rot_axis(y, -h_angle / 2.0f, dir, tmp); rot_axis(x, -v_angle / 2.0f, tmp, r00);
    rot_axis(y, h_angle / 2.0f, dir, tmp);  rot_axis(x, -v_angle / 2.0f, tmp, r10);
    rot_axis(y, -h_angle / 2.0f, dir, tmp); rot_axis(x, v_angle / 2.0f, tmp, r01);
    rot_axis(y, h_angle / 2.0f, dir, tmp);  rot_axis(x, v_angle / 2.0f, tmp, r11);
    for (int i = 0; i < 3; i++) {
        out_eye[i] = (float)eye[i];
        // Graphics::setView(eye, ray00, ray10, ray01, ray11): uniform ray01 <- camera ray10
        out_ray00[i] = (float)r00[i];
        out_ray01[i] = (float)r10[i];
        out_ray10[i] = (float)r01[i];
        out_ray11[i] = (float)r11[i];
    }
}

namespace {
// glReadPixels(GL_UNSIGNED_BYTE) of an RGBA32F texel: clamp, scale, round to nearest (even)
inline uint8_t to_unorm8(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 1.0f) return 255;
    return (uint8_t)std::nearbyint(f * 255.0f);
}
}  // namespace

extern "C" int rmr_encode_bmp(const float* rgba, int w, int h, const char* path) {
    if (!rgba || w <= 0 || h <= 0 || !path) return RMR_E_INVALID;
    std::vector<uint8_t> data((size_t)w * h * 4);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        for (int j = 0; j < 3; j++) {
            double c = (double)to_unorm8(rgba[i * 4 + j]) / 255.0;
            c = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);
            double s = (c <= 0.0031308) ? 12.92 * c : (1.0 + 0.055) * std::pow(c, 1.0 / 2.4);  // no -0.055
            s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s);
            data[i * 4 + j] = (uint8_t)(s * 255);
        }
        data[i * 4 + 3] = to_unorm8(rgba[i * 4 + 3]);
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return RMR_E_IO;
    const int pad = (-w * 3) & 3;
    const uint32_t img = (uint32_t)((w * 3 + pad) * h);
    uint8_t hdr[54] = {0};
    auto put16 = [&](int off, uint32_t v) { hdr[off] = v & 0xff; hdr[off + 1] = (v >> 8) & 0xff; };
    auto put32 = [&](int off, uint32_t v) { for (int k = 0; k < 4; k++) hdr[off + k] = (v >> (8 * k)) & 0xff; };
    hdr[0] = 'B'; hdr[1] = 'M';
    put32(2, 14 + 40 + img);
    put32(10, 14 + 40);
    put32(14, 40);
    put32(18, (uint32_t)w);
    put32(22, (uint32_t)h);
    put16(26, 1);
    put16(28, 24);
    std::fwrite(hdr, 1, 54, f);
    const uint8_t bg[3] = {255, 0, 255};
    std::vector<uint8_t> row((size_t)w * 3 + pad, 0);
    for (int y = h - 1; y >= 0; y--) {  // stb_image_write vdir = -1
        for (int x = 0; x < w; x++) {
            const uint8_t* d = &data[((size_t)y * w + x) * 4];
            int px[3];
            for (int k = 0; k < 3; k++) px[k] = bg[k] + ((d[k] - bg[k]) * d[3]) / 255;
            row[(size_t)x * 3 + 0] = (uint8_t)px[2];
            row[(size_t)x * 3 + 1] = (uint8_t)px[1];
            row[(size_t)x * 3 + 2] = (uint8_t)px[0];
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    return std::fclose(f) == 0 ? RMR_OK : RMR_E_IO;
}
