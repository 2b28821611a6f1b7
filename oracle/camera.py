"""oracle/camera.py — TEST INFRASTRUCTURE: restatement of Camera::calculateRays (Camera.cpp:25-102).

Vector3 is double (Vector.h:166-336); glm::mat3/vec3 are float; rotAxis builds
glm::mat3(0,-uz,uy, uz,0,-ux, -uy,ux,0), which is column-major, i.e. the transpose of the usual
cross-product matrix. numpy float32 scalars give IEEE single ops without FMA,
like MSVC 2013 /fp:precise SSE2 code.
"""
import math

import numpy as np

F = np.float32


def _f(x):
    return F(x)


def _cross(a, b):  # Vector3::cross, Vector.h:327-330 (double)
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _rot_axis(u, t, point):  # Camera.cpp:31-52 with origin (0,0,0)
    t = _f(t)
    ux, uy, uz = u
    uc = [[F(0), _f(-uz), _f(uy)], [_f(uz), F(0), _f(-ux)], [_f(-uy), _f(ux), F(0)]]  # columns
    ut = [[_f(ux * ux), _f(ux * uy), _f(ux * uz)], [_f(ux * uy), _f(uy * uy), _f(uy * uz)],
          [_f(ux * uz), _f(uy * uz), _f(uz * uz)]]
    c = _f(math.cos(float(t)))
    s = _f(math.sin(float(t)))
    omc = F(1) - c
    eye = [[F(1), F(0), F(0)], [F(0), F(1), F(0)], [F(0), F(0), F(1)]]
    R = [[(c * eye[j][i] + s * uc[j][i]) + omc * ut[j][i] for i in range(3)] for j in range(3)]
    v = [_f(point[0]), _f(point[1]), _f(point[2])]
    P = [R[0][i] * v[0] + R[1][i] * v[1] + R[2][i] * v[2] for i in range(3)]
    return (float(P[0]), float(P[1]), float(P[2]))


def calculate_rays(eye, direction, aspect, fov):
    """Returns camera-named (ray00, ray10, ray01, ray11) as double tuples."""
    aspect = _f(aspect)
    v_angle = _f(fov)
    h_angle = F(2) * _f(math.atan(float(aspect * _f(math.tan(float(v_angle / F(2)))))))
    z = tuple(float(x) for x in direction)
    x = _cross(z, (0.0, 1.0, 0.0))
    y = _cross(z, x)
    r00 = _rot_axis(x, -v_angle / F(2), _rot_axis(y, -h_angle / F(2), z))
    r10 = _rot_axis(x, -v_angle / F(2), _rot_axis(y, h_angle / F(2), z))
    r01 = _rot_axis(x, v_angle / F(2), _rot_axis(y, -h_angle / F(2), z))
    r11 = _rot_axis(x, v_angle / F(2), _rot_axis(y, h_angle / F(2), z))
    return r00, r10, r01, r11


def view_uniforms(eye, direction, aspect, fov):
    """The 15 floats uploaded by Graphics::setView, in shader-uniform order
    (eye, ray00, ray01, ray10, ray11) after Camera.cpp:101's argument swap."""
    r00, r10, r01, r11 = calculate_rays(eye, direction, aspect, fov)
    # setView(eye, ray00, ray10, ray01, ray11): uniform ray01 <- camera ray10, uniform ray10 <- camera ray01
    vals = list(eye) + list(r00) + list(r10) + list(r01) + list(r11)
    return np.array(vals, np.float32)


def default_view(W, H):
    """Program.cpp:102: Camera((0,4,-6), normalized(0,-3,6), W/H, PI/4) with PI = 3.141592653f."""
    d = (0.0, -3.0, 6.0)
    m = math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])
    d = (d[0] / m, d[1] / m, d[2] / m)
    pi = F(3.141592653)
    return view_uniforms((0.0, 4.0, -6.0), d, float(W) / float(H), pi / F(4))
