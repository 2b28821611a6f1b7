// Camera.cpp — the reference's Camera (Camera.cpp:1-179) over rmr_camera_view.
#include "Camera.h"

#include <cmath>

using Vector::Vector2;
using Vector::Vector3;

namespace {
// getLocal, Camera.cpp:25-29
void get_local(Vector3& x, Vector3& y, Vector3 z) {
    x = z.cross(Vector3(0, 1, 0));
    y = z.cross(x);
}

// rotAxis(u, t, point, origin), Camera.cpp:31-52: Rodrigues matrix in glm float arithmetic,
// applied to point - origin, origin added back.
Vector3 rot_axis(Vector3 u, float t, Vector3 point, Vector3 origin) {
    const float ux = (float)u.x, uy = (float)u.y, uz = (float)u.z;
    const float uc[3][3] = {{0.0f, -uz, uy}, {uz, 0.0f, -ux}, {-uy, ux, 0.0f}};  // columns
    const float ut[3][3] = {{(float)(u.x * u.x), (float)(u.x * u.y), (float)(u.x * u.z)},
                            {(float)(u.x * u.y), (float)(u.y * u.y), (float)(u.y * u.z)},
                            {(float)(u.x * u.z), (float)(u.y * u.z), (float)(u.z * u.z)}};
    const float c = std::cos(t), s = std::sin(t), omc = 1.0f - c;
    const float v[3] = {(float)(point.x - origin.x), (float)(point.y - origin.y), (float)(point.z - origin.z)};
    float p[3];
    for (int i = 0; i < 3; i++) {
        p[i] = 0.0f;
        float acc[3];
        for (int j = 0; j < 3; j++) acc[j] = (c * (i == j ? 1.0f : 0.0f) + s * uc[j][i]) + omc * ut[j][i];
        p[i] = acc[0] * v[0] + acc[1] * v[1] + acc[2] * v[2];
    }
    return Vector3(p[0] + origin.x, p[1] + origin.y, p[2] + origin.z);
}
}  // namespace

Camera::Camera() {}

Camera::Camera(Vector3 eyePos, Vector3 lookDir, float aspect_, float fov_) {
    aspect = aspect_;
    fov = fov_;
    eye = eyePos;
    dir = lookDir;
    calculateRays();
}

void Camera::calculateRays() {
    const double e[3] = {eye.x, eye.y, eye.z};
    const double d[3] = {dir.x, dir.y, dir.z};
    float oe[3], u00[3], u01[3], u10[3], u11[3];
    // rmr_camera_view returns shader-uniform order: uniform ray01 = the camera's ray10
    rmr_camera_view(e, d, aspect, fov, oe, u00, u01, u10, u11);
    ray00 = Vector3(u00[0], u00[1], u00[2]);
    ray10 = Vector3(u01[0], u01[1], u01[2]);
    ray01 = Vector3(u10[0], u10[1], u10[2]);
    ray11 = Vector3(u11[0], u11[1], u11[2]);
    if (Graphics::context()) Graphics::setView(eye, ray00, ray10, ray01, ray11);  // Camera.cpp:101
}

void Camera::zoom(float amount) {
    eye += dir * amount;
    calculateRays();
}

void Camera::pan(Vector2 amount) {
    Vector3 lx, ly;
    get_local(lx, ly, dir);
    eye += lx * amount.x;
    eye += ly * amount.y;
    calculateRays();
}

void Camera::orbit(Vector2 amount) {
    Vector3 lx, ly;
    get_local(lx, ly, dir);
    dir = rot_axis(ly, (float)amount.x, dir.normalized(), eye).normalized();
    dir = rot_axis(lx, (float)amount.y, dir.normalized(), eye).normalized();
    calculateRays();
}

void Camera::getRays(Vector3& r00, Vector3& r10, Vector3& r01, Vector3& r11) const {
    r00 = ray00;
    r10 = ray10;
    r01 = ray01;
    r11 = ray11;
}
