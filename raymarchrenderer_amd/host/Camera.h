// Camera.h — the reference's corner-ray camera (Camera.h:4-32). calculateRays() computes the four
// corner rays (Camera.cpp:54-102, via rmr_camera_view) and pushes them to Graphics::setView with
// the reference's argument order. update(sf::Window&) is replaced by the public zoom / pan /
// orbit controls it dispatched to (Camera.cpp:104-137); there is no window here.
#pragma once
#include "Graphics.h"
#include "Vector.h"

class Camera {
private:
    float aspect = 1.0f;
    float fov = 0.785398163f;
    Vector::Vector3 eye;
    Vector::Vector3 dir;
    Vector::Vector3 ray00, ray10, ray01, ray11;

public:
    Camera();
    Camera(Vector::Vector3 eyePos, Vector::Vector3 lookDir, float aspect, float fov);
    ~Camera() = default;
    void calculateRays();
    void setAspect(float newAspect) { aspect = newAspect; }
    void zoom(float amount);                  // Camera.cpp:104-109
    void pan(Vector::Vector2 amount);         // Camera.cpp:111-123
    void orbit(Vector::Vector2 amount);       // Camera.cpp:125-137
    Vector::Vector3 getEye() const { return eye; }
    Vector::Vector3 getDir() const { return dir; }
    // corner rays with the camera's own names (ray10 = +h, -v; ray01 = -h, +v)
    void getRays(Vector::Vector3& r00, Vector::Vector3& r10, Vector::Vector3& r01, Vector::Vector3& r11) const;
};
