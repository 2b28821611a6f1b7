// Vector.h — host vector types of the C++ facades (the reference's Vector.h namespace: double
// components, Vector2 / Vector3 / Vector4 with the arithmetic the host code uses).
#pragma once
#include <cmath>

namespace Vector {

struct Vector2 {
    double x = 0, y = 0;
    Vector2() = default;
    Vector2(double x_, double y_) : x(x_), y(y_) {}
    Vector2 operator+(Vector2 v) const { return {x + v.x, y + v.y}; }
    Vector2 operator-(Vector2 v) const { return {x - v.x, y - v.y}; }
    Vector2 operator*(double s) const { return {x * s, y * s}; }
    Vector2 operator/(double s) const { return {x / s, y / s}; }
    Vector2& operator+=(Vector2 v) { x += v.x; y += v.y; return *this; }
    bool operator==(Vector2 v) const { return x == v.x && y == v.y; }
    bool operator!=(Vector2 v) const { return !(*this == v); }
};

struct Vector3 {
    double x = 0, y = 0, z = 0;
    Vector3() = default;
    Vector3(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    Vector3 operator+(Vector3 v) const { return {x + v.x, y + v.y, z + v.z}; }
    Vector3 operator-(Vector3 v) const { return {x - v.x, y - v.y, z - v.z}; }
    Vector3 operator*(double s) const { return {x * s, y * s, z * s}; }
    Vector3 operator/(double s) const { return {x / s, y / s, z / s}; }
    Vector3& operator+=(Vector3 v) { x += v.x; y += v.y; z += v.z; return *this; }
    bool operator==(Vector3 v) const { return x == v.x && y == v.y && z == v.z; }
    double dot(Vector3 v) const { return x * v.x + y * v.y + z * v.z; }
    Vector3 cross(Vector3 v) const { return {y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x}; }
    double magnitude() const { return std::sqrt(x * x + y * y + z * z); }
    Vector3 normalized() const { double m = magnitude(); return m == 0 ? *this : *this / m; }
};

struct Vector4 {
    double x = 0, y = 0, z = 0, w = 0;
    Vector4() = default;
    Vector4(double x_, double y_, double z_, double w_) : x(x_), y(y_), z(z_), w(w_) {}
};

}  // namespace Vector
