// scene.hpp — scene JSON -> rmr tables (replaces the reference's GLSL code generator,
// Graphics.cpp:38-113 + 392-752).
#pragma once
#include <string>
#include <vector>
#include "../../include/rmr_tables.h"
#include "json.hpp"

namespace rmr {

struct SceneError : std::runtime_error {
    explicit SceneError(const std::string& m) : std::runtime_error(m) {}
};

struct CompiledScene {
    int variant = RMR_VARIANT_RM1;
    std::vector<rmr_prim> prims;
    std::vector<rmr_op> ops;
    std::vector<float> consts;          // xyz triples
    std::vector<rmr_material> materials;
    std::vector<rmr_spectral> spectral;
    rmr_spectral spectral_sky{};
    int v2_begin = 0, v2_end = 0, v2_slots = 0;
    rmr_rm2_consts rm2{};
    float sky[3] = {0.015f, 0.015f, 0.015f};

    rmr_scene view() const;                           // non-owning rmr_scene over the vectors
    void from_tables(const rmr_scene& s);             // deep copy
    double flops_per_map() const;
    double transc_per_map() const;                     // SURVEY §8d counting convention
};

// JSON text -> tables for `variant`; throws SceneError with the reason the reference's generated
// GLSL would fail to compile.
CompiledScene compile_scene(const std::string& json_text, int variant);
CompiledScene builtin_scene(int variant);
// largest |radius| of the scene's spheres (0 if none): the approximate-then-exact map's error scale
float max_sphere_radius(const CompiledScene& s);

}  // namespace rmr
